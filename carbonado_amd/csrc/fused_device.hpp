// fused_device.hpp — K13: encode() at Zfec|Bao in one pass (gfx950).
//
// encode() level 12 (encoding.rs:121-147) is zfec 4-of-8 of the object
// followed by bao over the zfec output.  Done as two kernels (K1-BL writes
// the shards into their chunk slots, K3 reads them back and hashes them) the
// 32 MiB of shards per 16 MiB object cross HBM twice.  Here one wave
// computes the shards of 8 consecutive chunk-columns and hashes the 64
// resulting chunks while they are still on chip:
//
//  * a wave's block = chunk-columns [ub, ub + 8) of one object = chunks
//    (shard sh, column u) for 8 shards x 8 columns.  The 8 steps of a block
//    each cover 128 B of every chunk.
//  * GF role (per step): lane (cu = lane/8, g = lane%8) loads 16 B of each of
//    the 4 data shards at column ub + cu, bytes 128 s + 16 g (coalesced: 8
//    lanes = one 128-B line), computes the 4 parity 16-B pieces with the
//    packed LDS table (one ds_read_b32 per input byte gives all 4 parity
//    products, as K1) and writes the 8 pieces into the LDS rows of chunks
//    (sh, cu) at word 4 g of the step's half-row.  The next step's loads are
//    issued after the stores, before the hashing (the next block's first
//    step at the last step), so they land while the lane compresses.
//  * store role: the 8 lanes of group cu store the stream lines of chunks
//    (t, cu), t = 0..7, whole 128-B memory lines read back from the rows (the
//    rows hold two steps, so the line ending at chunk byte d + 128 s is
//    complete at step s; bao K3 SP 3's path).
//  * hash role: lane L hashes row L = chunk (L/8, ub + L%8), two BLAKE3
//    compressions per step; after 8 steps its chunk CV goes to the level-0
//    CV buffer, from which the parent kernels (K4, K4t) build the tree and
//    write the parent nodes into the stream.
//
// HBM traffic per 16 MiB object: 16 MiB read + 32 MiB of chunk lines + the
// parents (2 MiB) and the 1 MiB of level-0 CVs written and read once — about
// 52 MiB against 84 MiB for K1-BL + K3.  The kernel is VALU-bound: 16
// compressions per chunk (672 lane-ops each) plus ~250 lane-ops of GF work
// per step.
#pragma once

#include "bao_device.hpp"
#include "zfec_device.hpp"

namespace chip {
namespace fused {

using bao::u32x2;
using bao::u32x4;

constexpr int FW = 8;               // waves per workgroup
constexpr int FTPB = 64 * FW;
constexpr int FR = 4;               // replicas of the GF table (4 data shards x FR dwords per byte value)
constexpr int RW = 68;              // LDS words per chunk row: [pad 4 | even step 32 | odd step 32]
constexpr size_t TAB_BYTES = 256 * 4 * FR * 4;
constexpr size_t LDS_BYTES = TAB_BYTES + (size_t)FW * 64 * RW * 4;  // 16 KiB + 136 KiB

struct FusedArgs {
    const uint8_t *in;
    uint64_t in_stride, valid, C;   // objects, bytes of data per object (zero beyond), shard length
    uint8_t *out;
    uint64_t out_stride;            // bao streams of the 8C-byte zfec outputs
    uint64_t count, N, cols, bpo;   // objects, chunks per stream, chunk-columns per shard, blocks per object
    const uint32_t *table;          // [4][256] packed parity products (4 parity rows per dword)
    const uint64_t *coff;           // [N] stream offset of each chunk (bao_chunk_table)
    uint8_t *cv;                    // level-0 CVs [count][N], or level-3 CVs [count][cvs] (FULL)
    uint32_t *queue;                // block queue (DQ): [0] next block, [32] waves done; zero at launch
    uint64_t cvs;                   // FULL: level-3 CVs per object = ceil(N / 8)
    uint8_t *cv3;                   // RT: level-3 CVs [count][cvs] (the groups the waves complete)
};

// RT (general path, runs of RT blocks): whether the aligned 8-chunk group g
// of a stream of 8 shards of `cols` chunk-columns each is completed inside a
// wave.  The group's chunks must lie in one shard t, at columns [u0, u0 + 8);
// its last column lies in block (u0 + 7) / 8, which completes it; the part
// before that block (u0 % 8 != 0: rows whose shard starts off the 8-chunk
// grid) lies in the previous block, processed by the same wave just before
// unless the completing block starts a run.  Everything else (groups across
// two shards, groups across a run boundary) is completed by the level-1-3
// pass from the level-0 CVs the waves store for exactly those chunks.
__host__ __device__ inline bool group_in_wave(uint64_t g, uint64_t cols, uint64_t bpo, uint64_t rt) {
    const uint64_t c0 = 8 * g, t = c0 / cols;
    if ((c0 + 7) / cols != t) return false;
    const uint64_t u0 = c0 - t * cols, b = (u0 + 7) / 8;
    if (b >= bpo) return false;
    return u0 % 8 == 0 || b % rt != 0;
}

__device__ __forceinline__ int dofs(int step) { return 4 + (step & 1) * 32; }

// LDS address of T[byte b of x] for table slot tb: byte * 64 + tb in two VALU
// ops for every b.  Written plainly, byte 0 compiles to shift, mask and add;
// the mask is kept opaque so that the shift and add fuse (v_lshl_add_u32).
__device__ __forceinline__ uint32_t gf_addr(uint32_t x, int b, uint32_t tb) {
    constexpr uint32_t ROWB = 4 * FR * 4;
    if (b == 0) {
        uint32_t t;
        asm("v_and_b32 %0, 0xff, %1" : "=v"(t) : "v"(x));
        return t * ROWB + tb;
    }
    return ((x >> (8 * b)) & 0xFFu) * ROWB + tb;
}

// The four table addresses of x's bytes in four VALU ops (GFP): the address
// pair of bytes 0 and 2 (hi = 0) or 1 and 3 (hi = 1) in one register, byte k
// times 64 in bits 6-13 / 22-29 and tb in both halves' low 6 bits, then split
// with a mask and a shift.  Per byte that is 1 VOP3 + 1.5 VOP2 against 2 VALU
// (one a VOP3, often both) for gf_addr.  The and-or is asm: written in C the
// compiler folds the halves back into per-byte extracts.
__device__ __forceinline__ uint32_t gf_pair(uint32_t x, int hi, uint32_t tb2) {
    const uint32_t sh = hi ? x >> 2 : x << 6;
    uint32_t t;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(t) : "v"(sh), "s"(0x3FC03FC0u), "v"(tb2));
    return t;
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, bao::glb(reinterpret_cast<u32x4 *>(p)));
    else *bao::glb(reinterpret_cast<u32x4 *>(p)) = v;
}

// Levels 1-3 of the tree inside the wave, pipelined over blocks.  With
// cols % 8 == 0 the 8 lanes 8j..8j+7 of a block hold the CVs of 8 aligned
// chunks of one shard: a complete subtree that is not the root (N >= 64).
// Its 7 parents need three dependent compressions; instead of three
// compression times per block (32, 16, 8 lanes busy) one step per block
// computes level 1 of this block (even lanes), level 2 of the previous block
// (lanes 4j+1, from the level-1 CVs lanes 4j and 4j+2 kept) and level 3 of
// the block before (lanes 8j+3, from lanes 8j+1 and 8j+5): 56 lanes, one
// compression.  Each parent node (l || r) is written at its stream slot —
// the node with leftmost chunk s at level k sits 64 k bytes before chunk s —
// and the level-3 CVs go to `cv` [count][N/8] for the parent kernels.
template <bool NT>
struct Tree {
    uint32_t pr[8];   // my last parent CV (roles 1 and 2)
    uint8_t *node;    // ... its node slot
    uint64_t cvi;     // ... global index (obj N + chunk) of its leftmost chunk
    bool ok = false;  // ... valid
    int lane;
    uint8_t *cv;
    bool wr = true;  // write the nodes (false: tools/fused_tune diagnostic DG 11)
    __device__ Tree(int l, uint8_t *c) : node(nullptr), cvi(0), lane(l), cv(c) {
#pragma unroll
        for (int w = 0; w < 8; ++w) pr[w] = 0u;
    }
    // h: my chunk CV; nd: the level-1 node slot of my chunk (even lanes);
    // gi: obj N + chunk; cur: this block has chunks (false when draining)
    __device__ __forceinline__ void step(const uint32_t (&h)[8], uint8_t *nd, uint64_t gi, bool cur) {
        const bool r1 = !(lane & 1), r2 = (lane & 3) == 1, r3 = (lane & 7) == 3;
        const int sl = r2 ? lane - 1 : lane - 2, sr = r2 ? lane + 1 : lane + 2;
        uint32_t l[8], r[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t hr = (uint32_t)__shfl_xor((int)h[w], 1);
            const uint32_t pl = (uint32_t)__shfl((int)pr[w], sl);
            const uint32_t pq = (uint32_t)__shfl((int)pr[w], sr);
            l[w] = r1 ? h[w] : pl;
            r[w] = r1 ? hr : pq;
        }
        const uint64_t tn = (uint64_t)__shfl((long long)(uintptr_t)node, sl);
        const uint64_t tc = (uint64_t)__shfl((long long)cvi, sl);
        const bool tok = __shfl((int)ok, sl) != 0;
        uint8_t *my = r1 ? nd : reinterpret_cast<uint8_t *>(tn) - 64;
        const uint64_t mc = r1 ? gi : tc;
        const bool act = r1 ? cur : ((r2 || r3) && tok);
        if (act) {
            uint32_t p[8];
            bao::b3_parent(l, r, false, p);
            if (wr) bao::node_io<0, NT>(my, l, r);
            if (r3) {
                bao::store_cv(cv + (mc / 8) * 32, p);
            } else {
#pragma unroll
                for (int w = 0; w < 8; ++w) pr[w] = p[w];
            }
        }
        node = my;
        cvi = mc;
        ok = act && !r3;
    }
};

// DG: diagnostics for tools/fused_tune (wrong output): 1 = no line stores,
// 2 = no hashing, 3 = no GF (rows get the data shards only), 4 = neither
// stores nor hashing, 5 = every chunk's lines 128-B aligned (no partial
// lines), 6 = 5 without hashing, 7 = the line stores' LDS reads without the
// stores, 8 = the whole-line stores aimed at 8 KiB per wave (L2 hits),
// 10 = GF table lookups without bank conflicts (wrong products); read-traffic
// attribution (tools/k13_fetch): 11 = FULL without the in-wave tree's node
// stores, 12 = general with the level 1-3 node slots in front of each chunk
// zero-filled at step 0 (lines whole inside the kernel), 13 = general without
// the level-0 CV stores, 14 = general with the level-0 CVs in a block-padded
// layout [obj][shard][8 bpo] (each block's 8 CVs of a shard = one aligned
// 256-B run).
// FULL: cols % 8 == 0 and no zfec padding (valid >= 4 C): every block is 8
// whole columns of plain loads, levels 1-3 run in the wave (Tree) and `cv`
// receives level-3 CVs; otherwise lanes are predicated and `cv` receives the
// level-0 CVs.  ORD 1 places the line stores between the step's two
// compressions (their LDS reads issued before the first) and the next step's
// loads after them; ORD 2 issues those loads first, as soon as the step's
// rows are written.
// KIND 0: encode() Zfec|Bao (zfec 4-of-8, then bao of the 8 shards); KIND 1:
// bao of the content itself (encoding::bao, encode() level 4; FULL only: the
// launch covers the whole 64-chunk blocks, bao_tail_kernel the rest).  KIND 1's block is 64 consecutive chunks (row / hash lane
// L = chunk ub + L), loaded 8 x 16 B per lane per step instead of computed.
// MP 1: both compressions' message words of a step are read from the rows at
// once, before the store role's piece reads, so the second compression's LDS
// reads land while the first one runs (MP 0: each read right before its
// compression, its latency exposed).
// SS 1: the step's 8 whole-line stores issued two after each of the first
// four rounds of the first compression (scheduling barriers around them)
// instead of as one burst between the compressions.
// O32: every object's input and stream are < 4 GiB (the host checks), so
// loads and stores address them as the wave's object base (SGPRs) plus a
// 32-bit per-lane offset: global_load/store with saddr, no 64-bit VALU adds
// per access.  GFP 1: table addresses through gf_pair.
// WPG: waves per workgroup (FW; tools/fused_tune runs 4 = one wave per SIMD
// to measure the kernel's sensitivity to occupancy).
//
// This is the kernel body; the product's launches are the few configurations
// fused_kernels.hip wraps in kernels of their own (zfec_bao_fused_kernel_full,
// _general, bao_content_fused_kernel), the tuner's are tools/fused_variants.hpp's.
template <bool NT, bool FULL, int ORD = 1, int DG = 0, int KIND = 0, bool DQ = true, int MP = 0, int SS = 0,
          bool O32 = false, int GFP = 0, int WPG = FW, bool NTL = false, int PRIO = 0, int RT = 0>
__device__ __forceinline__ void zfec_bao_fused_body(const FusedArgs &a) {
    static_assert(KIND == 0 || FULL, "content bao: FULL blocks only");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int NV = KIND ? 8 : 4;         // 16-B loads per lane per step
    constexpr uint64_t BW = KIND ? 64 : 8;   // chunks (KIND 1) / columns (KIND 0) per block
    const uint64_t TS = KIND ? 8 : a.cols;   // chunk index step between the 8 lane groups
    if (KIND == 0) {  // table: lds[x][s][r] = T_s[x], FR replicas
        uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
        for (int i = threadIdx.x; i < 256 * 4 * FR; i += 64 * WPG) {
            const int x = i / (4 * FR);
            const int s = (i - x * (4 * FR)) / FR;
            dst[i] = a.table[s * 256 + x];
        }
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    // WPG > FW (tools/fused_tune occupancy diagnostic only, wrong output): the
    // extra waves share the first waves' rows, the LDS holds FW waves' rows
    uint32_t *rows = reinterpret_cast<uint32_t *>(lds + TAB_BYTES) + (WPG > FW ? wave % FW : wave) * 64 * RW;
    const int rep = lane % FR, grp = (lane & 31) / FR;
    uint32_t tb[4], tb2[4];
    uint64_t ioff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // lane group grp walks the data shards in the rotated order (j + grp) mod 4
        tb[j] = (uint32_t)((((j + grp) & 3) * FR + rep) * 4);
        tb2[j] = tb[j] | (tb[j] << 16);
        ioff[j] = (uint64_t)((j + grp) & 3) * a.C;
    }
    const int gl = lane & 7, cu = lane >> 3;
    const uint64_t total = a.count * a.bpo;
    const uint64_t GW = (uint64_t)gridDim.x * WPG;

    // Loads of a step.  A block whose input columns all lie below `valid`
    // (every block of an object without zfec padding) takes plain loads whose
    // wait the compiler can defer to the first use; the masked form (a branch
    // and an immediate wait per load) only runs in an object's last blocks.
    auto load_step = [&](uint64_t blk, int s, u32x4 (&v)[NV]) {
        const uint64_t obj = blk / a.bpo, ub = (blk - obj * a.bpo) * BW;
        const uint8_t *ib = a.in + obj * a.in_stride;
        if (KIND == 1) {  // chunk ub + 8 t + cu, bytes 128 s + 16 gl
            if (O32) {
                const uint32_t o = (uint32_t)((ub + cu) * 1024) + 128u * s + 16u * gl;
#pragma unroll
                for (int t = 0; t < NV; ++t) {
                    const u32x4 *src = reinterpret_cast<const u32x4 *>(ib + (uint64_t)(o + 8192u * t));
                    v[t] = NTL ? __builtin_nontemporal_load(src) : *src;
                }
                return;
            }
            const uint8_t *b = ib + (ub + cu) * 1024 + 128 * (uint64_t)s + 16 * gl;
#pragma unroll
            for (int t = 0; t < NV; ++t) v[t] = *reinterpret_cast<const u32x4 *>(b + (uint64_t)t * 8192);
            return;
        }
        const uint64_t off = (ub + cu) * 1024 + 128 * (uint64_t)s + 16 * gl;
        const bool full = FULL || (ub + 8 <= a.cols && 3 * a.C + (ub + 8) * 1024 <= a.valid);  // wave-uniform
        if (full) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[j] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                                 ib + (O32 ? (uint64_t)((uint32_t)ioff[j] + (uint32_t)off) : ioff[j] + off)))
                     : O32 ? *reinterpret_cast<const u32x4 *>(ib + (uint64_t)((uint32_t)ioff[j] + (uint32_t)off))
                           : *reinterpret_cast<const u32x4 *>(ib + ioff[j] + off);
        } else if (KIND == 0) {
            const bool col = ub + cu < a.cols;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[j] = col ? zf::load16_masked(ib, ioff[j] + off, a.valid) : u32x4{0u, 0u, 0u, 0u};
        }
    };

    // RT > 0 (general path): the blocks come in runs of RT consecutive blocks of
    // one object (the queue hands out runs), so a wave holds each block's
    // predecessor and completes levels 1-3 of the aligned groups that start
    // in it (group_in_wave), as the FULL path does for all groups.  A tuner
    // variant (tools/k13_fetch), not shipped: 13 % slower kernel than RT = 0
    // at the level-15 shard length (profiles/r10e_session)
    constexpr bool RUNS = !FULL && RT > 0 && KIND == 0;
    Tree<NT> tree(lane, RUNS ? a.cv3 : a.cv);
    tree.wr = DG != 11;
    // Blocks: DQ takes them from a queue (one atomic per block and wave, lane
    // 0, vector memory), so waves on slower XCDs simply take fewer; otherwise
    // a static stride of GW.  The next block is known before the current one
    // starts, for its first loads at step 7.
    auto grab = [&]() -> uint64_t {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(a.queue, 1u);
        return (uint64_t)__builtin_amdgcn_readfirstlane(b);
    };
    const uint64_t rpo = RUNS ? (a.bpo + RT - 1) / RT : 1;  // runs per object
    uint64_t run_last = 0, srun = (uint64_t)blockIdx.x * WPG + wave;
    auto run_first = [&](uint64_t r) -> uint64_t {  // first block of run r (total: none left)
        if (r >= a.count * rpo) return total;
        const uint64_t o = r / rpo, b0 = o * a.bpo + (r - o * rpo) * RT;
        run_last = (b0 + RT < (o + 1) * a.bpo ? b0 + RT : (o + 1) * a.bpo) - 1;
        return b0;
    };
    auto next_block = [&](uint64_t b) -> uint64_t {
        if (RUNS) {
            if (b < run_last) return b + 1;
            if (!DQ) srun += GW;
            return run_first(DQ ? grab() : srun);
        }
        return DQ ? grab() : b + GW;
    };
    uint64_t blk = RUNS ? run_first(DQ ? grab() : srun) : DQ ? grab() : (uint64_t)blockIdx.x * WPG + wave;
    uint32_t hp[8];  // RUNS: the previous block's chunk CVs
#pragma unroll
    for (int w = 0; w < 8; ++w) hp[w] = 0u;
    u32x4 v[NV], v2[NV];  // this step's loads; ORD 3: the next step's too
    if (blk < total) {
        load_step(blk, 0, v);
        if (ORD == 3) load_step(blk, 1, v2);
    }
    for (uint64_t nxt; blk < total; blk = nxt) {
        nxt = next_block(blk);
        const uint64_t obj = blk / a.bpo, ub = (blk - obj * a.bpo) * BW;
        uint8_t *ob = a.out + obj * a.out_stride;
        if (ub == 0 && lane == 0)  // u64 LE content length
            *bao::glb(reinterpret_cast<uint64_t *>(ob)) = KIND ? a.valid : 8 * a.C;
        const bool gcol = FULL || ub + cu < a.cols;         // store role: chunks (t, ub + cu)
        const uint64_t hu = ub + (lane & 7);                // hash role: chunk (lane / 8, hu)
        const bool mine = FULL || hu < a.cols;
        const uint64_t ci = (uint64_t)(lane >> 3) * TS + hu;
        const uint64_t hco = FULL ? a.coff[ci] : 0;          // tree role: my chunk's stream offset
        uint8_t *lsp[8];   // !O32: chunk (t, ub + cu)'s slot
        uint32_t lso[8];   // O32: its offset in the stream
        uint32_t ldd[8];
        {
            uint64_t co[8];  // all 8 offset loads in flight together
            const uint64_t c0 = gcol ? ub + cu : 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) co[t] = a.coff[(uint64_t)t * TS + c0];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                uint8_t *p = ob + co[t];
                if (DG == 5 || DG == 6) p = reinterpret_cast<uint8_t *>((uintptr_t)p & ~(uintptr_t)127);
                ldd[t] = (DG == 5 || DG == 6) ? 0u : (uint32_t)(-(uintptr_t)p) & 127u;
                if (O32) lso[t] = (uint32_t)(p - ob);
                else lsp[t] = p;
            }
        }
        auto lat = [&](int t, uint32_t x) -> uint8_t * {
            return O32 ? ob + (uint64_t)(lso[t] + x) : lsp[t] + x;
        };
        // head/tail stores (steps 0 and 7): their offsets do not depend on the
        // step, and hoisted out of the step loop they become 24 64-bit
        // addresses held across it (+17 VGPRs); the empty asm keeps each one
        // computed where it is used, folded into the store's saddr form
        auto lat_ht = [&](int t, uint32_t x) -> uint8_t * {
            if (!O32) return lsp[t] + x;
            uint32_t o = lso[t] + x;
            asm volatile("" : "+v"(o));
            return ob + (uint64_t)o;
        };
        uint32_t h[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) h[w] = bao::IV(w);

        for (int s = 0; s < 8; ++s) {
            // PRIO 1 (tools/fused_tune): the GF and store roles at raised wave
            // priority, the compressions at the base one
            if (PRIO) __builtin_amdgcn_s_setprio(1);
            // ---- GF role: 8 pieces of 16 B into the rows of chunks (sh, cu) ----
            if (KIND == 1) {  // content: the 8 loaded pieces are the rows' bytes
                const int wo = dofs(s) + 4 * gl;
#pragma unroll
                for (int t = 0; t < NV; ++t) *reinterpret_cast<u32x4 *>(rows + (t * 8 + cu) * RW + wo) = v[t];
            } else {
            uint32_t acc[16];
            if (DG == 3) {
#pragma unroll
                for (int c = 0; c < 16; ++c) acc[c] = zf::comp(v[c & 3], c >> 2);
            } else {
                // per output word, the 4 shards' lookups together: independent
                // LDS reads the compiler can keep in flight (shard-outer order
                // left it one register for them, an lgkmcnt(0) per lookup)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t x[4], ad[4][4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        x[j] = zf::comp(v[j], d);
                        // DG 10 (diagnostic, wrong bytes): lanes l and l + 16 look up
                        // table rows of opposite parity, so no two lanes of a 32-lane
                        // half meet on one bank (FR 4: bank = 16 (x & 1) + 4 s + r)
                        if (DG == 10) x[j] = (x[j] & 0xFEFEFEFEu) | ((uint32_t)((lane >> 4) & 1) * 0x01010101u);
                        if (GFP) {
                            const uint32_t t02 = gf_pair(x[j], 0, tb2[j]), t13 = gf_pair(x[j], 1, tb2[j]);
                            ad[j][0] = t02 & 0xFFFFu; ad[j][2] = t02 >> 16;
                            ad[j][1] = t13 & 0xFFFFu; ad[j][3] = t13 >> 16;
                        }
                    }
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        uint32_t e[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            e[j] = *reinterpret_cast<const uint32_t *>(lds + (GFP ? ad[j][b] : gf_addr(x[j], b, tb[j])));
                        // v_bitop3 (gfx950): three of the four terms in one instruction
                        acc[d * 4 + b] = __builtin_amdgcn_bitop3_b32(e[0], e[1], e[2], 0x96) ^ e[3];
                    }
                }
            }
            const int wo = dofs(s) + 4 * gl;
#pragma unroll
            for (int j = 0; j < 4; ++j)  // v[j] is data shard (j + grp) mod 4
                *reinterpret_cast<u32x4 *>(rows + (((j + grp) & 3) * 8 + cu) * RW + wo) = v[j];
            {
                u32x4 p[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t r0, r1, r2, r3;
                    zf::transpose4(acc[d * 4 + 0], acc[d * 4 + 1], acc[d * 4 + 2], acc[d * 4 + 3], r0, r1, r2, r3);
                    if (d == 0) { p[0].x = r0; p[1].x = r1; p[2].x = r2; p[3].x = r3; }
                    if (d == 1) { p[0].y = r0; p[1].y = r1; p[2].y = r2; p[3].y = r3; }
                    if (d == 2) { p[0].z = r0; p[1].z = r1; p[2].z = r2; p[3].z = r3; }
                    if (d == 3) { p[0].w = r0; p[1].w = r1; p[2].w = r2; p[3].w = r3; }
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) *reinterpret_cast<u32x4 *>(rows + ((4 + q) * 8 + cu) * RW + wo) = p[q];
            }
            }
            bao::wave_sync();

            auto next_loads = [&]() {
                if (s < 7) load_step(blk, s + 1, v);
                else if (nxt < total) load_step(nxt, 0, v);
            };
            if (ORD == 2) next_loads();  // as soon as v is free: two compressions of cover
            if (ORD == 3) {  // two steps ahead: v takes the next step's data, v2 loads the one after
#pragma unroll
                for (int t = 0; t < NV; ++t) v[t] = v2[t];
                if (s < 6) load_step(blk, s + 2, v2);
                else if (nxt < total) load_step(nxt, s - 6, v2);
            }

            // ---- store role: whole 128-B memory lines of chunks (t, cu) ----
            // 8 B at chunk byte x (x % 8 == 0): the row's two step halves are one
            // 256-B ring after the 16-B pad, so byte x sits at pad + x mod 256
            // (= dofs(x >> 7) + (x & 127) / 4 words, in two VALU ops)
            auto piece = [&](const uint32_t *row, uint32_t x) -> u32x2 {
                return *reinterpret_cast<const u32x2 *>(reinterpret_cast<const uint8_t *>(row) + 16 + (x & 255u));
            };
            auto read_msg = [&](int hh, uint32_t (&m)[16]) {
                const u32x4 *r = reinterpret_cast<const u32x4 *>(rows + lane * RW + dofs(s) + hh * 16);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const u32x4 x = r[q4];
                    m[4 * q4] = x.x; m[4 * q4 + 1] = x.y; m[4 * q4 + 2] = x.z; m[4 * q4 + 3] = x.w;
                }
            };
            constexpr bool HS = DG != 2 && DG != 4 && DG != 6;  // hashing on
            uint32_t mA[16], mB[16];
            if (MP && HS && mine) {
                read_msg(0, mA);
                read_msg(1, mB);
            }
            constexpr bool ST = DG != 1 && DG != 4;
            u32x4 q[8];
            if (ST && s >= 1) {  // the whole line [d + 128 (s-1), d + 128 s) of every chunk
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const uint32_t x = ldd[t] + 128u * (s - 1) + 16u * gl;
                    const uint32_t *row = rows + (t * 8 + cu) * RW;
                    const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                    q[t] = u32x4{lo.x, lo.y, hi.x, hi.y};
                }
            }
            auto one_line = [&](int t) {
                if (DG == 8)  // diagnostic: the same stores into 8 KiB per wave (L2-resident)
                    st16<NT>(a.out + ((uint64_t)(blockIdx.x * WPG + wave) * 8192 + t * 1024 + lane * 16), q[t]);
                else
                    st16<NT>(lat(t, ldd[t] + 128u * (s - 1) + 16u * gl), q[t]);
            };
            auto line_stores = [&]() {
                if (ST && s >= 1 && gcol && !SS) {
                    if (DG == 7) {  // diagnostic: the piece reads without the line stores
#pragma unroll
                        for (int t = 0; t < 8; ++t) h[7] ^= q[t].x ^ q[t].w;
                    } else {
#pragma unroll
                        for (int t = 0; t < 8; ++t) one_line(t);
                    }
                }
                if (DG == 12 && s == 0 && gcol) {  // zero the level 1-3 node slots in front of each chunk
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const uint64_t c = (uint64_t)t * TS + ub + cu;
                        uint32_t k = 0;
                        for (uint32_t l = 1; l <= 3; ++l)
                            if (c % (1ull << l) == 0 && c + (1ull << (l - 1)) < a.N) k = l;
                        for (uint32_t i = gl; i < 8 * k; i += 8)
                            *bao::glb(reinterpret_cast<u32x2 *>(lat_ht(t, 8 * i) - 64 * k)) = u32x2{0u, 0u};
                    }
                }
                if (ST && (s == 0 || s == 7) && gcol) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const uint32_t d = ldd[t];
                        const uint32_t *row = rows + (t * 8 + cu) * RW;
                        if (s == 0) {  // head [0, d)
                            const uint32_t hd = d & 8u;
                            if (hd && gl == 0) *bao::glb(reinterpret_cast<u32x2 *>(lat_ht(t, 0))) = piece(row, 0);
                            const uint32_t x = 16u * gl + hd;
                            if (x + 16 <= d) {
                                const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                                *bao::glb(reinterpret_cast<u32x4 *>(lat_ht(t, x))) = u32x4{lo.x, lo.y, hi.x, hi.y};
                            }
                        } else {  // tail [896 + d, 1024)
                            const uint32_t x = 896u + d + 16u * gl;
                            if (x + 16 <= 1024) {
                                const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                                *bao::glb(reinterpret_cast<u32x4 *>(lat_ht(t, x))) = u32x4{lo.x, lo.y, hi.x, hi.y};
                            } else if (x + 8 == 1024) {
                                *bao::glb(reinterpret_cast<u32x2 *>(lat_ht(t, x))) = piece(row, x);
                            }
                        }
                    }
                }
                // next loads, after this step's stores, in flight during the compressions
                if (ORD <= 1) next_loads();
            };

            // ---- hash role: blocks 2s, 2s+1 of my chunk ----
            auto hash = [&](int hh) {
                if (!HS) {  // keep the rows' reads alive
                    h[hh] ^= rows[lane * RW + dofs(s) + hh];
                } else if (mine) {
                    const int b = 2 * s + hh;
                    const uint32_t flags = (b == 0 ? bao::F_CHUNK_START : 0u) | (b == 15 ? bao::F_CHUNK_END : 0u);
                    if (SS && hh == 0) {
                        uint32_t m[16];
                        if (MP) {
#pragma unroll
                            for (int w = 0; w < 16; ++w) m[w] = mA[w];
                        } else {
                            read_msg(0, m);
                        }
                        const bool do_st = ST && s >= 1 && gcol && DG != 7;
                        bao::b3_compress_cb(h, m, ci, 64, flags, [&](int r) {
                            if (r < 4 && do_st) {
                                __builtin_amdgcn_sched_barrier(0);
                                one_line(2 * r);
                                one_line(2 * r + 1);
                                __builtin_amdgcn_sched_barrier(0);
                            }
                        });
                    } else if (MP) {
                        bao::b3_compress(h, hh ? mB : mA, ci, 64, flags);
                    } else {
                        uint32_t m[16];
                        read_msg(hh, m);
                        bao::b3_compress(h, m, ci, 64, flags);
                    }
                }
            };
            if (ORD >= 1) {
                if (PRIO) __builtin_amdgcn_s_setprio(0);
                hash(0);
                if (PRIO) __builtin_amdgcn_s_setprio(1);
                line_stores();
                if (PRIO) __builtin_amdgcn_s_setprio(0);
                hash(1);
            } else {
                line_stores();
                hash(0);
                hash(1);
            }
            bao::wave_sync();
        }
        if (FULL) {
            tree.step(h, ob + hco - 64, obj * 8 * a.cvs + ci, true);
        } else if (RUNS) {
            // row t's aligned group that this block completes: columns [ub - d, ub - d + 8),
            // element j held by lane 8t + ((j - d) & 7) of this block (j >= d) or of the
            // previous one (j < d), d = the row's offset from the 8-chunk grid
            const int t = lane >> 3, j = lane & 7;
            const uint32_t d = (uint32_t)(((uint64_t)t * a.cols) & 7);
            const uint64_t gc0 = (uint64_t)t * a.cols + ub - d;  // its first chunk
            const bool ok = ub >= d && group_in_wave(gc0 / 8, a.cols, a.bpo, RT);
            const int src = (lane & ~7) | ((j - (int)d) & 7);
            uint32_t g[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const uint32_t x = (uint32_t)__shfl((int)h[w], src), y = (uint32_t)__shfl((int)hp[w], src);
                g[w] = j >= (int)d ? x : y;
                hp[w] = h[w];
            }
            const uint64_t ec = gc0 + j;  // my element's chunk
            tree.step(g, ob + (ok ? a.coff[ec] : 64) - 64, obj * 8 * a.cvs + ec, ok);
            // my own chunk's level-0 CV when its group is left to the level-1-3 pass
            if (mine && !group_in_wave(ci / 8, a.cols, a.bpo, RT)) {
                auto *cvp = bao::glb(reinterpret_cast<u32x4 *>(a.cv + (obj * a.N + ci) * 32));
                cvp[0] = u32x4{h[0], h[1], h[2], h[3]};
                cvp[1] = u32x4{h[4], h[5], h[6], h[7]};
            }
        } else if (mine && DG != 13) {
            const uint64_t cvi = DG == 14 ? obj * 8 * (8 * a.bpo) + (uint64_t)(lane >> 3) * (8 * a.bpo) + hu
                                          : obj * a.N + ci;
            auto *cvp = bao::glb(reinterpret_cast<u32x4 *>(a.cv + cvi * 32));
            cvp[0] = u32x4{h[0], h[1], h[2], h[3]};
            cvp[1] = u32x4{h[4], h[5], h[6], h[7]};
        }
    }
    if (FULL || RUNS) {  // drain: level 2 of the last block, level 3 of the last two
        uint32_t z[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        tree.step(z, nullptr, 0, false);
        tree.step(z, nullptr, 0, false);
    }
    if (DQ && lane == 0) {  // the last wave out leaves the queue zero for the next launch
        const uint32_t done = atomicAdd(a.queue + 32, 1u);
        if (done + 1 == gridDim.x * (uint32_t)WPG) {
            a.queue[0] = 0u;
            a.queue[32] = 0u;
        }
    }
}

// The last chunks of a content-mode bao encode (encode() level 4, bao of the
// content) whose chunk count is not a multiple of 64: KIND 1 covers the whole
// 64-chunk blocks [0, Nf) of every object, this kernel the rest [Nf, N), at
// most 64 chunks including a short last chunk: one wave per object, one lane
// per chunk, content read and copied into the chunk's slot straight from
// memory (a few KiB per object), levels 1-3 of the tail's aligned 8-chunk
// groups merged through lane shuffles with bao's promotion rule (a node
// without a right child is its left child), nodes written at their slots and
// the level-3 CVs stored beside KIND 1's for the parent kernels (from level
// 4).  N > 64, so none of these nodes is the root.
struct TailArgs {
    const uint8_t *in;
    uint64_t in_stride, n;
    uint8_t *out;
    uint64_t out_stride;
    uint64_t count, N, Nf, cvs;
    const uint64_t *coff;  // [N] stream offset of each chunk
    uint8_t *cv;           // level-3 CVs [count][cvs]
};

__global__ __launch_bounds__(64) void bao_tail_kernel(TailArgs a) {
    const uint64_t obj = blockIdx.x;
    const int lane = threadIdx.x;
    const uint64_t ci = a.Nf + (uint64_t)lane;
    const bool on = obj < a.count && ci < a.N;
    const uint8_t *src = a.in + obj * a.in_stride + ci * 1024;
    uint8_t *ob = a.out + obj * a.out_stride;
    uint32_t h[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) h[w] = bao::IV(w);
    if (on) {
        const uint64_t rem = a.n - ci * 1024;
        const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;  // >= 1: ci < N = ceil(n / 1024)
        const uint32_t nb = (clen + 63) / 64;
        uint8_t *dst = ob + a.coff[ci];  // 8-B aligned slot
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t blen = clen - 64 * b < 64 ? clen - 64 * b : 64u;
            uint32_t m[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t off = 64 * b + 16 * q;
                const uint32_t valid = off < clen ? clen - off : 0u;
                const u32x4 x = valid >= 16 ? *reinterpret_cast<const u32x4 *>(src + off)
                                            : bao::load16_partial(src + off, valid);
                m[4 * q] = x.x; m[4 * q + 1] = x.y; m[4 * q + 2] = x.z; m[4 * q + 3] = x.w;
                if (valid >= 16) bao::store16_a8<false>(dst + off, x);
                else if (valid) bao::store16_partial(dst + off, x, valid);
            }
            const uint32_t flags = (b == 0 ? bao::F_CHUNK_START : 0u) | (b + 1 == nb ? bao::F_CHUNK_END : 0u);
            bao::b3_compress(h, m, ci, blen, flags);
        }
    }
#pragma unroll
    for (int L = 1; L <= 3; ++L) {
        const int d = 1 << (L - 1);
        uint32_t r[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) r[w] = (uint32_t)__shfl((int)h[w], (lane + d) & 63);
        if (on && (lane & (2 * d - 1)) == 0 && ci + d < a.N) {  // a real node: both children exist
            uint32_t p[8];
            bao::node_io<0, false>(ob + bao::parent_stream_off(ci, L, a.N), h, r);
            bao::b3_parent(h, r, false, p);
#pragma unroll
            for (int w = 0; w < 8; ++w) h[w] = p[w];
        }
    }
    if (on && (lane & 7) == 0) bao::store_cv(a.cv + (obj * a.cvs + ci / 8) * 32, h);
}

// Levels 1-3 of the tree from the chunk CVs, for the streams the kernel's
// FULL path does not cover (8 does not divide the shard's chunk count, e.g.
// level 15's 4097-chunk shards, or zfec padding): one lane per aligned group
// of 8 chunks [8g, 8g + 8), its up to 7 parents computed one after another
// with bao's promotion rule (a node without a right child is its left child),
// each real node written at its slot (64 l bytes before its leftmost chunk),
// the level-3 CV stored for the parent kernels, which start at level 4.
// N > 8, so none of these nodes is the root.  (Three K4 launches with a CV
// round trip per level did this before: ~2.1 ms per 1024 x 16 MiB step.)
// NW: how the nodes are written (tools/fused_tune A/B): 1 = eight 8-B stores,
// 2 = four 16-B stores (8-B aligned), 0 = not at all (diagnostic).
template <int NW = 1>
__global__ __launch_bounds__(256) void bao_levels123_kernel(const uint8_t *cv0, uint64_t N, uint64_t count,
                                                            const uint64_t *coff, uint8_t *out, uint64_t out_stride,
                                                            uint8_t *cv3, uint64_t n3) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= count * n3) return;
    const uint64_t obj = gid / n3, g = gid - obj * n3, s0 = 8 * g;
    const uint32_t cnt = N - s0 < 8 ? (uint32_t)(N - s0) : 8u;
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
    uint8_t *ob = out + obj * out_stride;
#pragma unroll
    for (int l = 1; l <= 3; ++l) {
        const uint32_t span = 1u << l, half = span >> 1;  // chunks per node at level l, and per child
#pragma unroll
        for (int q = 0; q < (8 >> l); ++q) {
            const uint32_t left = q * span;       // first chunk of node q (group-relative)
            const int li = q * 2, ri = q * 2 + 1;  // child slots at level l - 1
            if (left + half < cnt) {  // a real node: both children exist
                uint8_t *node = ob + coff[s0 + left] - 64 * l;
                if (NW == 1) bao::node_io<0, false>(node, c[li], c[ri]);
                if (NW == 2) {
                    auto *q4 = (__attribute__((address_space(1))) bao::u32x4_a8 *)node;
                    q4[0] = bao::u32x4_a8{c[li][0], c[li][1], c[li][2], c[li][3]};
                    q4[1] = bao::u32x4_a8{c[li][4], c[li][5], c[li][6], c[li][7]};
                    q4[2] = bao::u32x4_a8{c[ri][0], c[ri][1], c[ri][2], c[ri][3]};
                    q4[3] = bao::u32x4_a8{c[ri][4], c[ri][5], c[ri][6], c[ri][7]};
                }
                uint32_t p[8];
                bao::b3_parent(c[li], c[ri], false, p);
#pragma unroll
                for (int w = 0; w < 8; ++w) c[q][w] = p[w];
            } else {  // promoted (or empty): the left child
#pragma unroll
                for (int w = 0; w < 8; ++w) c[q][w] = c[li][w];
            }
        }
    }
    bao::store_cv(cv3 + (obj * n3 + g) * 32, c[0]);
}

// The same with the node stores coalesced (NW 3): one wave per block; the
// nodes go to LDS first, then the wave writes them four lanes per node, 16
// nodes (64 contiguous bytes each) per store instruction instead of 64 lanes
// at 64 places 8 KiB apart.  QS: nodes per lane staged at once (4: a whole
// level, 16 KiB of LDS per wave; 1: node by node, 4 KiB, so LDS no longer
// caps the waves per CU below what the registers allow).
// rt > 0: only the groups K13's run mode left (group_in_wave false; cols,
// bpo: the zfec shards' chunk-columns and K13's blocks per object).
// L > 0: levels L+1..L+3 from the N level-L CVs per object in cv0 (the same
// groups of 8 one level-L stride up: a level-(L+l) node whose leftmost chunk
// is c sits 64 (L + l) bytes before chunk c, its left spine being complete),
// for the top of many small trees (fused_kernels.hip upper_levels); N > 8.
template <int QS>
__global__ __launch_bounds__(64) void bao_levels123_lds_kernel(const uint8_t *cv0, uint64_t N, uint64_t count,
                                                               const uint64_t *coff, uint8_t *out,
                                                               uint64_t out_stride, uint8_t *cv3, uint64_t n3,
                                                               uint64_t cols = 0, uint64_t bpo = 0, uint64_t rt = 0,
                                                               uint32_t L = 0) {
    __shared__ bao::u32x4 buf[64 * QS * 4];  // [lane][node][16-B unit] of the nodes staged
    __shared__ uint64_t naddr[64 * QS];      // [lane][node]: its slot (0: not a real node)
    const int lane = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * 64 + lane;
    bool on = gid < count * n3;
    const uint64_t obj = on ? gid / n3 : 0, g = on ? gid - obj * n3 : 0, s0 = 8 * g;
    if (rt && on && group_in_wave(g, cols, bpo, rt)) on = false;  // completed in K13's wave
    const uint32_t cnt = !on ? 0u : (N - s0 < 8 ? (uint32_t)(N - s0) : 8u);
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
    uint8_t *ob = out + obj * out_stride;
#pragma unroll
    for (int l = 1; l <= 3; ++l) {
        const uint32_t span = 1u << l, half = span >> 1;
#pragma unroll
        for (int q0 = 0; q0 < (8 >> l); q0 += QS) {
            const int ns = (8 >> l) - q0 < QS ? (8 >> l) - q0 : QS;  // nodes per lane this round
#pragma unroll
            for (int j = 0; j < ns; ++j) {
                const int q = q0 + j;
                const uint32_t left = q * span;
                const int li = q * 2, ri = q * 2 + 1;
                const bool real = left + half < cnt;
                bao::u32x4 *b = buf + (lane * ns + j) * 4;
                b[0] = bao::u32x4{c[li][0], c[li][1], c[li][2], c[li][3]};
                b[1] = bao::u32x4{c[li][4], c[li][5], c[li][6], c[li][7]};
                b[2] = bao::u32x4{c[ri][0], c[ri][1], c[ri][2], c[ri][3]};
                b[3] = bao::u32x4{c[ri][4], c[ri][5], c[ri][6], c[ri][7]};
                naddr[lane * ns + j] =
                    real ? (uint64_t)(uintptr_t)(ob + coff[(s0 + left) << L] - 64 * (L + l)) : 0ull;
                if (real) {
                    uint32_t p[8];
                    bao::b3_parent(c[li], c[ri], false, p);
#pragma unroll
                    for (int w = 0; w < 8; ++w) c[q][w] = p[w];
                } else {
#pragma unroll
                    for (int w = 0; w < 8; ++w) c[q][w] = c[li][w];
                }
            }
            bao::wave_sync();
            for (int i = 0; i < ns * 4; ++i) {  // unit k = i * 64 + lane: node k / 4, 16-B unit k % 4
                const int k = i * 64 + lane;
                const uint64_t a = naddr[k >> 2];
                if (a) *(__attribute__((address_space(1))) bao::u32x4_a8 *)(uintptr_t)(a + 16 * (k & 3)) =
                    bao::u32x4_a8{buf[k].x, buf[k].y, buf[k].z, buf[k].w};
            }
            bao::wave_sync();
        }
    }
    if (on) bao::store_cv(cv3 + (obj * n3 + g) * 32, c[0]);
}

}  // namespace fused
}  // namespace chip
