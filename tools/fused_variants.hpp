// fused_variants.hpp — the tuner's K13 kernels (any configuration of the body)
// and measured-and-not-kept variants of the fused kernels, for tools/ only
// (not part of the library):
//  * K13S, zfec_bao_spec_kernel: K13's FULL path with hashing and GF/line
//    stores on separate waves (profiles/NOT_KEPT.md, r7jk: 15-20 % slower);
//  * bao_levels123_seg_kernel: the general path's levels-1-3 pass writing
//    whole 64-B segments (profiles/r7q: 0.499 vs 0.380 ms per 256 objects).
#pragma once

#include "../carbonado_amd/csrc/fused_device.hpp"

namespace chip {
namespace fused {

// The tuner's K13 variants: any configuration of the kernel body
// (fused_device.hpp zfec_bao_fused_body documents the arguments), each its
// own kernel.  The library instantiates only the configurations it ships
// (fused_kernels.hip: zfec_bao_fused_kernel_full / _general, ...).
template <bool NT, bool FULL, int ORD = 1, int DG = 0, int KIND = 0, bool DQ = true, int MP = 0, int SS = 0,
          bool O32 = false, int GFP = 0, int WPG = FW, bool NTL = false, int PRIO = 0, int RT = 0>
__global__ __launch_bounds__(64 * WPG) void zfec_bao_fused_kernel(FusedArgs a) {
    zfec_bao_fused_body<NT, FULL, ORD, DG, KIND, DQ, MP, SS, O32, GFP, WPG, NTL, PRIO, RT>(a);
}

// K13S (tools/fused_tune only; measured 15-20 % SLOWER than K13, profiles/r7j,
// r7k, not in the library): the FULL path of K13 with its roles on different
// waves.  The lockstep the per-step barrier imposes costs more than the
// overlap gains: the producers, with a third or a quarter of their SIMD's
// issue slots, hold the hash waves at every barrier.  In K13
// every wave alternates between GF work (table lookups with LDS round trips,
// loads, whole-line stores) and hashing, and only two waves fit a SIMD (rows
// and 232 VGPRs), so the stalls of one wave's GF phase are hidden only when
// the other wave happens to be hashing.  Here a workgroup of 12 waves (three
// per SIMD) has 8 hash waves, each with its own 8-column block and rows as in
// K13, and 4 producer waves, producer p computing the shards of hash waves
// 2p and 2p+1 and writing their stream lines.  The rows are the same ping-pong
// pair of step halves; one s_barrier per step hands a step from producers to
// hashers: during step s the hashers compress step s (half s & 1) while the
// producers store the lines complete at step s and then write step s + 1 into
// the other half, whose step s - 1 those line stores were the last to read.
// Blocks go to the workgroup eight at a time (a group, one queue atomic),
// the next group's id taken one group ahead so that the producers can fill
// its first step during the current group's last.  LDS: the same 16 KiB
// table + 8 x 17 KiB of rows as K13.
constexpr int SHW = 8;                 // hash waves per workgroup
// NPB: hash waves (blocks) per producer wave: 2 = 12-wave workgroups (3 per
// SIMD), 1 = 16-wave workgroups (4 per SIMD, <= 128 VGPRs)
template <int NPB> constexpr int stpb() { return 64 * (SHW + SHW / NPB); }
constexpr int STPB = 64 * (SHW + SHW / 2);
constexpr size_t S_LDS_BYTES = TAB_BYTES + (size_t)SHW * 64 * RW * 4 + 16;

template <bool NT, int NPB = 2>
__global__ __launch_bounds__(stpb<NPB>()) void zfec_bao_spec_kernel(FusedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    {
        uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
        for (int i = threadIdx.x; i < 256 * 4 * FR; i += stpb<NPB>()) {
            const int x = i / (4 * FR);
            const int sh = (i - x * (4 * FR)) / FR;
            dst[i] = a.table[sh * 256 + x];
        }
    }
    uint32_t *gslot = reinterpret_cast<uint32_t *>(lds + TAB_BYTES + (size_t)SHW * 64 * RW * 4);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const bool hasher = wave < SHW;
    const uint64_t total = a.count * a.bpo;
    const uint64_t ngroups = (total + SHW - 1) / SHW;
    // ---- producer state: blocks 2p, 2p + 1 of the group ----
    const int pw = wave - SHW;
    const int rep = lane % FR, grp = (lane & 31) / FR;
    const int gl = lane & 7, cu = lane >> 3;
    uint32_t tb2[4], ioff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t tb = (uint32_t)((((j + grp) & 3) * FR + rep) * 4);
        tb2[j] = tb | (tb << 16);
        ioff[j] = (uint32_t)(((j + grp) & 3) * a.C);
    }
    auto rows_of = [&](int h) -> uint32_t * { return reinterpret_cast<uint32_t *>(lds + TAB_BYTES) + h * 64 * RW; };
    // global step q = 8 * (group ordinal) + s; producers load step q + 2 and compute step q + 1
    auto load_blk = [&](uint64_t blk, int st, u32x4 (&v)[4]) {
        if (blk >= total) return;
        const uint64_t obj = blk / a.bpo, ub = (blk - obj * a.bpo) * 8;
        const uint8_t *ib = a.in + obj * a.in_stride;
        const uint32_t off = (uint32_t)((ub + cu) * 1024) + 128u * st + 16u * gl;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const u32x4 *>(ib + (uint64_t)(ioff[j] + off));
    };
    auto gf_rows = [&](uint64_t blk, int st, const u32x4 (&v)[4], uint32_t *rows) {
        if (blk >= total) return;
        uint32_t acc[16];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t ad[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t x = zf::comp(v[j], d);
                const uint32_t t02 = gf_pair(x, 0, tb2[j]), t13 = gf_pair(x, 1, tb2[j]);
                ad[j][0] = t02 & 0xFFFFu; ad[j][2] = t02 >> 16;
                ad[j][1] = t13 & 0xFFFFu; ad[j][3] = t13 >> 16;
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                uint32_t e[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) e[j] = *reinterpret_cast<const uint32_t *>(lds + ad[j][b]);
                acc[d * 4 + b] = __builtin_amdgcn_bitop3_b32(e[0], e[1], e[2], 0x96) ^ e[3];
            }
        }
        const int wo = dofs(st) + 4 * gl;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<u32x4 *>(rows + (((j + grp) & 3) * 8 + cu) * RW + wo) = v[j];
        u32x4 pq[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t r0, r1, r2, r3;
            zf::transpose4(acc[d * 4 + 0], acc[d * 4 + 1], acc[d * 4 + 2], acc[d * 4 + 3], r0, r1, r2, r3);
            if (d == 0) { pq[0].x = r0; pq[1].x = r1; pq[2].x = r2; pq[3].x = r3; }
            if (d == 1) { pq[0].y = r0; pq[1].y = r1; pq[2].y = r2; pq[3].y = r3; }
            if (d == 2) { pq[0].z = r0; pq[1].z = r1; pq[2].z = r2; pq[3].z = r3; }
            if (d == 3) { pq[0].w = r0; pq[1].w = r1; pq[2].w = r2; pq[3].w = r3; }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<u32x4 *>(rows + ((4 + q) * 8 + cu) * RW + wo) = pq[q];
    };
    // per block: stream offsets of chunks (t, ub + cu); their line phases are
    // derived where used (two VALU) rather than held (8 VGPRs a block)
    struct Lines { uint32_t lso[8]; uint8_t *ob; bool on; };
    auto lines_of = [&](uint64_t blk, Lines &L) {
        L.on = blk < total;
        if (!L.on) return;
        const uint64_t obj = blk / a.bpo, ub = (blk - obj * a.bpo) * 8;
        L.ob = a.out + obj * a.out_stride;
        uint64_t co[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) co[t] = a.coff[(uint64_t)t * a.cols + ub + cu];
#pragma unroll
        for (int t = 0; t < 8; ++t) L.lso[t] = (uint32_t)co[t];
        if (ub == 0 && lane == 0) *bao::glb(reinterpret_cast<uint64_t *>(L.ob)) = 8 * a.C;  // u64 LE length
    };
    auto piece = [](const uint32_t *row, uint32_t x) -> u32x2 {
        return *reinterpret_cast<const u32x2 *>(reinterpret_cast<const uint8_t *>(row) + 16 + (x & 255u));
    };
    auto store_lines = [&](const Lines &L, const uint32_t *rows, int st) {
        if (!L.on) return;
        const uint32_t ob_lo = (uint32_t)(uintptr_t)L.ob;
        auto at = [&](int t, uint32_t x) -> uint8_t * {
            uint32_t o = L.lso[t] + x;
            asm volatile("" : "+v"(o));
            return L.ob + (uint64_t)o;
        };
        if (st >= 1) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t d = (0u - ob_lo - L.lso[t]) & 127u;
                const uint32_t x = d + 128u * (st - 1) + 16u * gl;
                const uint32_t *row = rows + (t * 8 + cu) * RW;
                const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                st16<NT>(L.ob + (uint64_t)(L.lso[t] + x), u32x4{lo.x, lo.y, hi.x, hi.y});
            }
        }
        if (st == 0 || st == 7) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t d = (0u - ob_lo - L.lso[t]) & 127u;
                const uint32_t *row = rows + (t * 8 + cu) * RW;
                if (st == 0) {  // head [0, d)
                    const uint32_t hd = d & 8u;
                    if (hd && gl == 0) *bao::glb(reinterpret_cast<u32x2 *>(at(t, 0))) = piece(row, 0);
                    const uint32_t x = 16u * gl + hd;
                    if (x + 16 <= d) {
                        const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                        *bao::glb(reinterpret_cast<u32x4 *>(at(t, x))) = u32x4{lo.x, lo.y, hi.x, hi.y};
                    }
                } else {  // tail [896 + d, 1024)
                    const uint32_t x = 896u + d + 16u * gl;
                    if (x + 16 <= 1024) {
                        const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                        *bao::glb(reinterpret_cast<u32x4 *>(at(t, x))) = u32x4{lo.x, lo.y, hi.x, hi.y};
                    } else if (x + 8 == 1024) {
                        *bao::glb(reinterpret_cast<u32x2 *>(at(t, x))) = piece(row, x);
                    }
                }
            }
        }
    };

    Tree<NT> tree(lane, a.cv);
    uint32_t *hrows = rows_of(hasher ? wave : 0);
    uint32_t *rX[NPB];
    u32x4 vX[NPB][4];
    Lines LX[NPB];
#pragma unroll
    for (int x = 0; x < NPB; ++x) {
        rX[x] = rows_of(hasher ? 0 : NPB * pw + x);
        LX[x].on = false;
    }
    // The iterations run over global steps q: group ordinal q / 8 (0 is a
    // virtual group before the first, whose step 7 only lets the producers
    // fill the first group's step 0), step s = q % 8.  Group ordinal k grabs
    // ordinal k + 1's id at its step 0 into slot (k + 1) & 1, read after the
    // step's barrier.
    if (threadIdx.x == 0) gslot[1] = atomicAdd(a.queue, 1u);
    __syncthreads();
    uint64_t cur = ngroups, nxt = gslot[1];
    if (!hasher && nxt < ngroups) {
#pragma unroll
        for (int x = 0; x < NPB; ++x) load_blk(nxt * SHW + NPB * pw + x, 0, vX[x]);
    }
    uint64_t obj = 0, ci = 0, hco = 0;
    uint8_t *ob = nullptr;
    bool hon = false;
    uint32_t h[8];
    for (uint64_t q = 7;; ++q) {
        const int s = (int)(q & 7);
        if (s == 0) {
            cur = nxt;
            if (cur >= ngroups) break;
            if (threadIdx.x == 0) gslot[((q >> 3) + 1) & 1] = atomicAdd(a.queue, 1u);
            const uint64_t blk = cur * SHW + wave;
            hon = hasher && blk < total;
            if (hon) {  // my block's chunk (lane / 8, ub + lane % 8)
                obj = blk / a.bpo;
                const uint64_t ub = (blk - obj * a.bpo) * 8;
                ob = a.out + obj * a.out_stride;
                ci = (uint64_t)(lane >> 3) * a.cols + ub + (lane & 7);
                hco = a.coff[ci];
            }
#pragma unroll
            for (int w = 0; w < 8; ++w) h[w] = bao::IV(w);
        }
        if (s == 1) nxt = gslot[((q >> 3) + 1) & 1];
        if (hasher) {
            if (hon) {
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    uint32_t m[16];
                    const u32x4 *r = reinterpret_cast<const u32x4 *>(hrows + lane * RW + dofs(s) + hh * 16);
#pragma unroll
                    for (int q4 = 0; q4 < 4; ++q4) {
                        const u32x4 x = r[q4];
                        m[4 * q4] = x.x; m[4 * q4 + 1] = x.y; m[4 * q4 + 2] = x.z; m[4 * q4 + 3] = x.w;
                    }
                    const int b = 2 * s + hh;
                    const uint32_t flags = (b == 0 ? bao::F_CHUNK_START : 0u) | (b == 15 ? bao::F_CHUNK_END : 0u);
                    bao::b3_compress(h, m, ci, 64, flags);
                }
            }
            if (s == 7 && cur < ngroups) tree.step(h, hon ? ob + hco - 64 : nullptr, obj * 8 * a.cvs + ci, hon);
        } else {
#pragma unroll
            for (int x = 0; x < NPB; ++x) store_lines(LX[x], rX[x], s);
            // step s + 1 (the next group's step 0 at s = 7) into its half
            const uint64_t gA = (s == 7 ? nxt : cur) * SHW + NPB * pw;
#pragma unroll
            for (int x = 0; x < NPB; ++x) gf_rows(gA + x, (s + 1) & 7, vX[x], rX[x]);
            // loads of step s + 2 (the next group's steps 0 and 1 at s = 6, 7)
            const uint64_t lA = (s < 6 ? cur : nxt) * SHW + NPB * pw;
#pragma unroll
            for (int x = 0; x < NPB; ++x) load_blk(lA + x, (s + 2) & 7, vX[x]);
            if (s == 7) {
#pragma unroll
                for (int x = 0; x < NPB; ++x) lines_of(gA + x, LX[x]);
            }
        }
        __syncthreads();
    }
    if (hasher) {  // drain: level 2 of the last block, level 3 of the last two
        uint32_t z[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        tree.step(z, nullptr, 0, false);
        tree.step(z, nullptr, 0, false);
    }
    if (threadIdx.x == 0) {  // the last workgroup out leaves the queue zero for the next launch
        const uint32_t done = atomicAdd(a.queue + 32, 1u);
        if (done + 1 == gridDim.x) {
            a.queue[0] = 0u;
            a.queue[32] = 0u;
        }
    }
}

// The same pass writing whole 64-B memory segments (SEG).  Node slots sit at
// 8 (mod 64), so every node written alone leaves two partial segments whose
// other bytes (chunk bytes K13 wrote, neighbouring nodes) were written long
// before: 3.1 GB of segment writes for 2.0 GB of nodes (profiles/r6l).  Here
// the nodes in front of one chunk are written as one stack — [L3 L2 L1]
// before chunk 8g, [L2 L1] before 8g + 4, [L1] before 8g + 2 and 8g + 6 —
// widened to whole segments with the 8 bytes before the stack and the
// chunk's first 56 bytes, read back from the stream and written unchanged
// (K13 has finished; bytes of a higher node that K4 writes later are
// rewritten by K4).  Stacks of different chunks touch disjoint segments.
// Groups with fewer than 8 chunks (a stream's last) take the per-node path.
template <int K>  // nodes in the stack
__device__ __forceinline__ void seg_stack(uint8_t *ob, uint64_t chunk_off, const uint32_t (*nodes)[16]) {
    // region [chunk_off - 64 K - 8, chunk_off + 56): 64-B aligned, K + 1 segments
    uint8_t *base = ob + chunk_off - 64 * K - 8;
    uint32_t w[16 * (K + 1)];
    const u32x2 pre = *bao::glb(reinterpret_cast<const u32x2 *>(base));
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const u32x2 x = *bao::glb(reinterpret_cast<const u32x2 *>(ob + chunk_off + 8 * q));
        w[2 + 16 * K + 2 * q] = x.x;
        w[3 + 16 * K + 2 * q] = x.y;
    }
    w[0] = pre.x;
    w[1] = pre.y;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) w[2 + 16 * k + i] = nodes[k][i];
    auto *q4 = bao::glb(reinterpret_cast<u32x4 *>(base));
#pragma unroll
    for (int i = 0; i < 4 * (K + 1); ++i) q4[i] = u32x4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
}

__global__ __launch_bounds__(256) void bao_levels123_seg_kernel(const uint8_t *cv0, uint64_t N, uint64_t count,
                                                                const uint64_t *coff, uint8_t *out,
                                                                uint64_t out_stride, uint8_t *cv3, uint64_t n3) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= count * n3) return;
    const uint64_t obj = gid / n3, g = gid - obj * n3, s0 = 8 * g;
    const uint32_t cnt = N - s0 < 8 ? (uint32_t)(N - s0) : 8u;
    uint8_t *ob = out + obj * out_stride;
    if (cnt < 8) {  // the stream's last group: the per-node path (bao's promotion rule)
        uint32_t c[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if ((uint32_t)i < cnt) {
                bao::load_cv(cv0 + (obj * N + s0 + i) * 32, c[i]);
            } else {
#pragma unroll
                for (int w = 0; w < 8; ++w) c[i][w] = 0u;
            }
        }
#pragma unroll
        for (int l = 1; l <= 3; ++l) {
            const uint32_t span = 1u << l, half = span >> 1;
#pragma unroll
            for (int q = 0; q < (8 >> l); ++q) {
                const uint32_t left = q * span;
                const int li = q * 2, ri = q * 2 + 1;
                if (left + half < cnt) {
                    bao::node_io<0, false>(ob + coff[s0 + left] - 64 * l, c[li], c[ri]);
                    uint32_t p[8];
                    bao::b3_parent(c[li], c[ri], false, p);
#pragma unroll
                    for (int w = 0; w < 8; ++w) c[q][w] = p[w];
                } else {
#pragma unroll
                    for (int w = 0; w < 8; ++w) c[q][w] = c[li][w];
                }
            }
        }
        bao::store_cv(cv3 + (obj * n3 + g) * 32, c[0]);
        return;
    }
    uint32_t c0[8][8];  // level-0 CVs
#pragma unroll
    for (int i = 0; i < 8; ++i) bao::load_cv(cv0 + (obj * N + s0 + i) * 32, c0[i]);
    uint32_t n1[4][16], p1[4][8];  // level-1 nodes (children) and CVs
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int w = 0; w < 8; ++w) { n1[q][w] = c0[2 * q][w]; n1[q][8 + w] = c0[2 * q + 1][w]; }
        bao::b3_parent(c0[2 * q], c0[2 * q + 1], false, p1[q]);
    }
    seg_stack<1>(ob, coff[s0 + 2], &n1[1]);
    seg_stack<1>(ob, coff[s0 + 6], &n1[3]);
    uint32_t n2[2][16], p2[2][8];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
        for (int w = 0; w < 8; ++w) { n2[q][w] = p1[2 * q][w]; n2[q][8 + w] = p1[2 * q + 1][w]; }
        bao::b3_parent(p1[2 * q], p1[2 * q + 1], false, p2[q]);
    }
    {
        uint32_t st[2][16];
#pragma unroll
        for (int i = 0; i < 16; ++i) { st[0][i] = n2[1][i]; st[1][i] = n1[2][i]; }
        seg_stack<2>(ob, coff[s0 + 4], st);
    }
    uint32_t n3n[16], p3[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) { n3n[w] = p2[0][w]; n3n[8 + w] = p2[1][w]; }
    bao::b3_parent(p2[0], p2[1], false, p3);
    {
        uint32_t st[3][16];
#pragma unroll
        for (int i = 0; i < 16; ++i) { st[0][i] = n3n[i]; st[1][i] = n2[0][i]; st[2][i] = n1[0][i]; }
        seg_stack<3>(ob, coff[s0], st);
    }
    bao::store_cv(cv3 + (obj * n3 + g) * 32, p3);
}

}  // namespace fused
}  // namespace chip
