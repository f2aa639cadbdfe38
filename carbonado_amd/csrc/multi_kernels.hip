// multi_kernels.hip — KM: one single object's bao stream over many
// workgroups, for latency (gfx950).
//
// A single object's encode()/decode() is the reference's real unit (segments
// of at most ~1 MB, README.md:107-111).  Of the two paths before KM, K13 /
// K3 give one lane a whole 1 KiB chunk (16 dependent compressions of ~700
// VALU): a 1 MiB object at Zfec|Bao is 2048 lanes = 32 waves on a 1024-SIMD
// chip, 65-115 us of kernel, and its tree top another 15-23 us launch
// (profiles/r10zm_session, r11a); KS (small_kernels.hip) puts a quad of lanes
// on each compression but one workgroup on the object, so it stops at 512
// chunks.  KM is KS spread over the chip:
//
//  * workgroup g (256 threads = 64 quads) owns the aligned group of 64 chunks
//    [64 g, 64 g + 64): one quad per chunk computes its CV (four lanes per
//    compression, quad_b3.hpp), then the group's own parent levels 1-6 (its
//    subtree; the pairing with the odd last node promoted is bao's
//    left-balanced tree, and group boundaries are aligned at every level <= 6)
//    are hashed from LDS and stored (encode) or compared with the stored nodes
//    (decode);
//  * each group's level-6 CV goes to global scratch; the workgroup that
//    finishes last (an agent-scope counter, released / acquired with fences:
//    the eight XCDs' L2s are not coherent without them) walks levels 7 ..
//    root over the G group CVs in LDS, four lanes per parent, and writes the
//    root hash (encode) or checks it against the expected one (decode).  It
//    resets the counter for the stream's next launch.
//
// Chunk bytes come from a contiguous source for chunks below `n_in` (bao of
// the content: the content itself) and from the stream's chunk slots above it
// (Zfec|Bao: every shard, written by parity_kernel<0>; decode: the stream).
// For a single call from host memory (api_single.cpp) the source, the stream
// to verify, the expected hash and every output live in pinned host memory:
// the kernels read and write them over PCIe themselves (zero-copy), so no
// DMA hop and no copy-engine-to-kernel handoff (~10-14 us each, r11c) sits
// on the call's critical path.  Encode writes the parent nodes in front of
// the first `nd` chunks compactly (`nodes`) and the rest into the stream's
// image from t0 on (`tail`); the host writes the chunks it holds itself.
#include "bao_device.hpp"
#include "chip_internal.hpp"
#include "quad_b3.hpp"
#include "zfec_device.hpp"

#include <cstdlib>
#include <cstring>

namespace chip {

using namespace bao;

namespace multi {

constexpr int TPB = 256, QUADS = TPB / 4;  // 64 quads per workgroup
constexpr int S = 64;                      // chunks per workgroup (the default SG; at most QUADS)
constexpr int GMAX = (int)(KM_MAX_N / S);  // groups the last workgroup's walk holds in LDS

struct MultiArgs {
    const uint8_t *src;    // chunks [0, n_in): contiguous source (zero past `valid`)
    const uint8_t *stream; // chunks [n_in, N) in their slots; decode: the whole stream (nodes too)
    uint8_t *out;          // decode: content bytes [0, out_limit) (null: verify only)
    uint8_t *nodes;        // encode: compact copy of the nodes in front of chunks [0, nd) (null: none)
    uint8_t *tail;         // encode: the stream image from byte t0 on, the other nodes land there (null: none)
    uint64_t t0;
    uint64_t n, N;         // bao content bytes and chunks
    uint64_t n_in, valid;  // source chunks, source bytes
    uint64_t nd, out_limit;
    uint8_t *hash;         // encode: root hash out; decode: expected
    uint32_t *status;      // decode: 0 or CHIP_ERR_BAO_HASH_MISMATCH (zero at launch)
    uint8_t *gcv;          // [G][32] group CVs
    uint32_t *counter;     // zero at launch; the last workgroup resets it
};

// the 64-B node (l || r) of parent P at `level`: my 16 B are words 4q .. 4q+3
__device__ __forceinline__ void node_out(const MultiArgs &a, uint64_t P, int level, int q, u32x4 mw) {
    const uint64_t s = P << level, off = parent_stream_off(s, level, a.N);
    if (s < a.nd) {
        if (a.nodes) store16_a8<false>(a.nodes + (off - 8 - 1024 * s) + 16 * q, mw);
    } else if (a.tail) {
        store16_a8<false>(a.tail + (off - a.t0) + 16 * q, mw);
    }
}

// Phase 4 of the KM kernels: publish this group's CV (word t of it in lanes
// 0-7: `mycv`); the workgroup that finishes last walks levels LOGS + 1 ..
// root over the G group CVs in `cv` (LDS [2][GMAX][8]), decode checking the
// top's stored nodes staged in `stored` (LDS, GMAX * 4 x 16 B).
template <int MODE, int LOGS>
__device__ __forceinline__ void km_top(const MultiArgs &a, uint32_t mycv, uint32_t (*cv)[GMAX][8], u32x4 *stored,
                                       uint32_t &last, const uint8_t *mbase, uint32_t (*msg)[16],
                                       const small::MsgIdx &mi, uint32_t iv0, uint32_t iv1) {
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const uint64_t grp = blockIdx.x, G = gridDim.x, N = a.N;
    if (t < 8) *glb(reinterpret_cast<uint32_t *>(a.gcv + grp * 32) + t) = mycv;
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // my group CV (and nodes) before the count
        const uint32_t done = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = done + 1 == (uint32_t)G;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every group's CV visible to every lane
    for (uint64_t i = t; i < 8 * G; i += TPB)
        cv[0][i >> 3][i & 7] = __hip_atomic_load(reinterpret_cast<const uint32_t *>(a.gcv) + i, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (MODE == 1) {  // level by level: pairs floor(cnt / 2), 16 B per lane of a quad
        uint64_t cnt = G, base = 0;
        for (int level = LOGS + 1; cnt > 1; ++level) {
            const uint64_t pairs = cnt / 2;
            for (uint64_t i = t; i < 4 * pairs; i += TPB)
                stored[4 * base + i] = load16_a8(a.stream + parent_stream_off((i >> 2) << level, level, N) + 16 * (i & 3));
            base += pairs;
            cnt = (cnt + 1) / 2;
        }
    }
    __syncthreads();
    uint64_t nbase = 0;  // decode: index of this level's first node in `stored`
    int cur = 0;
    uint64_t cnt_prev = G;
    bool ok = true;
    for (int level = LOGS + 1; cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        for (uint64_t p = g; p < cnt; p += QUADS) {
            if (2 * p + 1 >= cnt_prev) {
                cv[cur ^ 1][p][q] = cv[cur][2 * p][q];
                cv[cur ^ 1][p][4 + q] = cv[cur][2 * p][4 + q];
                continue;
            }
            const u32x4 mw = *reinterpret_cast<const u32x4 *>(&cv[cur][2 * p + (q >> 1)][4 * (q & 1)]);
            *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = mw;
            wave_sync();
            const bool root = cnt == 1;
            uint32_t h0 = iv0, h1 = iv1;
            small::compress4(h0, h1, mbase, mi, q, iv0, 0, 64, F_PARENT | (root ? F_ROOT : 0u));
            wave_sync();
            if (MODE == 0) {
                node_out(a, p, level, q, mw);
            } else {
                const u32x4 s = stored[4 * (nbase + p) + q];
                ok &= s.x == mw.x && s.y == mw.y && s.z == mw.z && s.w == mw.w;
            }
            if (root) {
                uint32_t *hp = reinterpret_cast<uint32_t *>(a.hash);
                if (MODE == 0) {
                    hp[q] = h0;
                    hp[4 + q] = h1;
                } else {
                    ok &= hp[q] == h0 && hp[4 + q] == h1;
                }
            } else {
                cv[cur ^ 1][p][q] = h0;
                cv[cur ^ 1][p][4 + q] = h1;
            }
        }
        __syncthreads();
        cur ^= 1;
        nbase += cnt_prev / 2;
        cnt_prev = cnt;
    }
    if (MODE == 1 && !ok) flag_mismatch(a.status, 0);
}

// SG chunks per workgroup (a power of two <= QUADS; fewer spreads a small
// object's loads over more CUs, the top walk then starts lower)
template <int MODE, int SG>
__global__ __launch_bounds__(TPB) void km_kernel(MultiArgs a) {
    constexpr int LOGS = SG == 64 ? 6 : SG == 32 ? 5 : SG == 16 ? 4 : -1;
    static_assert(LOGS > 0, "SG: 16, 32 or 64");
    __shared__ __attribute__((aligned(16))) uint32_t cvs[2][GMAX][8];  // a level and the next
    __shared__ __attribute__((aligned(16))) uint32_t msg[QUADS][16];   // each quad's message block
    __shared__ uint32_t last;
    __shared__ __attribute__((aligned(16))) u32x4 stored[MODE == 1 ? GMAX * 4 : 4];  // decode: the top's nodes
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const uint64_t grp = blockIdx.x, N = a.N, n = a.n;
    const uint64_t c0 = grp * SG, r = N - c0 < (uint64_t)SG ? N - c0 : (uint64_t)SG;  // my chunks
    bool ok = true;

    // ---- phase 1 (decode): the header checked, content bytes out
    if (MODE == 1) {
        if (grp == 0 && t == 0 && *reinterpret_cast<const uint64_t *>(a.stream) != n) ok = false;
        const uint64_t lim = a.out ? (a.out_limit < (c0 + r) * 1024 ? a.out_limit : (c0 + r) * 1024) : 0;
        for (uint64_t o = c0 * 1024 + 16 * (uint64_t)t; o < lim; o += 16 * TPB) {
            const uint8_t *p = a.stream + chunk_stream_off(o / 1024, N) + o % 1024;
            const uint64_t left = lim - o;
            if (left >= 16) *glb(reinterpret_cast<u32x4 *>(a.out + o)) = load16_a8(p);
            else store16_partial(a.out + o, load16_partial(p, (uint32_t)left), (uint32_t)left);
        }
    }

    // ---- phase 2: chunk CVs, one quad per chunk
    const uint32_t slot = (uint32_t)(reinterpret_cast<uintptr_t>(&msg[g][0]) - reinterpret_cast<uintptr_t>(&msg[0][0]));
    const uint8_t *mbase = reinterpret_cast<const uint8_t *>(&msg[0][0]);
    const small::MsgIdx mi(q, slot);
    const uint32_t iv0 = q == 0 ? IV(0) : q == 1 ? IV(1) : q == 2 ? IV(2) : IV(3);
    const uint32_t iv1 = q == 0 ? IV(4) : q == 1 ? IV(5) : q == 2 ? IV(6) : IV(7);
    u32x4 stn[LOGS];  // decode: stored nodes (a zero-copy stream costs a PCIe round trip per load)
    if ((uint64_t)g < r) {
        const uint64_t c = c0 + g;
        const uint64_t rem = n - c * 1024;
        const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
        const uint32_t nb = (clen + 63) / 64;  // N >= 2: every chunk holds at least one byte
        const bool from_src = c < a.n_in;
        const uint8_t *cp = a.stream + chunk_stream_off(c, N);
        if (MODE == 1) {  // the stored nodes this quad checks at levels 1 .. LOGS, in flight with the chunk
            uint64_t cp_ = r;
#pragma unroll
            for (int l = 1; l <= LOGS; ++l) {
                const uint64_t cn = (cp_ + 1) / 2;
                if ((uint64_t)g < cn && 2 * (uint64_t)g + 1 < cp_)
                    stn[l - 1] = load16_a8(a.stream + parent_stream_off(((c0 >> l) + g) << l, l, N) + 16 * q);
                cp_ = cn;
            }
        }
        u32x4 pc[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) {  // my 16 B of every block of the chunk, all loads in flight
            const uint32_t off = 64 * b + 16 * q;
            if (off >= clen) pc[b] = u32x4{0u, 0u, 0u, 0u};
            else if (from_src) pc[b] = zf::load16_masked(a.src, c * 1024 + off, a.valid);
            else pc[b] = off + 16 <= clen ? load16_a8(cp + off) : small::load16_bytes(cp + off, clen - off);
        }
        uint32_t h0 = iv0, h1 = iv1;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            if ((uint32_t)b < nb) {
                *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = pc[b];
                wave_sync();
                const bool lastb = (uint32_t)b + 1 == nb;
                const uint32_t flags = (b == 0 ? F_CHUNK_START : 0u) | (lastb ? F_CHUNK_END : 0u);
                small::compress4(h0, h1, mbase, mi, q, iv0, c, lastb ? clen - 64 * b : 64u, flags);
                wave_sync();
            }
        }
        cvs[0][g][q] = h0;
        cvs[0][g][4 + q] = h1;
    }
    __syncthreads();

    // ---- phase 3: the group's levels 1 .. LOGS, one quad per parent
    int cur = 0;
    uint64_t cnt_prev = r;
    for (int level = 1; level <= LOGS && cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        if ((uint64_t)g < cnt) {
            const uint64_t p = g;
            if (2 * p + 1 >= cnt_prev) {  // odd last node: promoted unchanged
                cvs[cur ^ 1][p][q] = cvs[cur][2 * p][q];
                cvs[cur ^ 1][p][4 + q] = cvs[cur][2 * p][4 + q];
            } else {
                const u32x4 mw = *reinterpret_cast<const u32x4 *>(&cvs[cur][2 * p + (q >> 1)][4 * (q & 1)]);
                *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = mw;
                wave_sync();
                uint32_t h0 = iv0, h1 = iv1;
                small::compress4(h0, h1, mbase, mi, q, iv0, 0, 64, F_PARENT);
                wave_sync();
                const uint64_t P = (c0 >> level) + p;
                if (MODE == 0) {
                    node_out(a, P, level, q, mw);
                } else {
                    u32x4 s = stn[0];
#pragma unroll
                    for (int l = 2; l <= LOGS; ++l)
                        if (level == l) s = stn[l - 1];
                    ok &= s.x == mw.x && s.y == mw.y && s.z == mw.z && s.w == mw.w;
                }
                cvs[cur ^ 1][p][q] = h0;
                cvs[cur ^ 1][p][4 + q] = h1;
            }
        }
        __syncthreads();
        cur ^= 1;
        cnt_prev = cnt;
    }
    if (MODE == 1 && !ok) flag_mismatch(a.status, 0);

    // ---- phase 4: publish the group CV; the last workgroup walks the top
    km_top<MODE, LOGS>(a, t < 8 ? cvs[cur][0][t] : 0u, cvs, stored, last, mbase, msg, mi, iv0, iv1);
}

// ---- KM with each workgroup's range staged in LDS ----------------------------
// km_kernel's quads load 16 B of each 64-B block of their chunk: a chunk's 16
// loads sit 64 B apart and a wave's 16 chunks 1 KiB apart.  Over PCIe from
// pinned host memory that pattern reads a 2.2 MB stream at ~39 GB/s, whole
// contiguous rows at ~49 (tools/bar_probe, profiles/r11_session/r11v/r11t_bar.log).
// So where the chunks come from pinned memory -- decode (the stream) and bao
// of the content (the content) -- each workgroup first copies its contiguous
// range into LDS, 4 KiB per instruction across the workgroup: decode, the
// group's region of the stream (its left-spine nodes, then its chunks and
// nodes in pre-order: 64 chunks + 63 nodes = 69,568 B for a full group);
// encode, its 64 KiB of content.  The quads hash their chunks from LDS and
// decode checks the group's stored nodes there; the top walk's buffers reuse
// the staging area once the group's levels are done.  Same bytes and verdicts
// as km_kernel (CHIP_KM_STAGE=0 keeps km_kernel for the A/B).
constexpr int STAGE_VEC = 17;  // 16-B loads per lane
static_assert(STAGE_VEC * TPB * 16 >= 64 * 1024 + 63 * 64 + 15, "a group's stream region and its alignment slack");
static_assert(STAGE_VEC * TPB * 16 >= 2 * GMAX * 32 + GMAX * 64, "the top walk's CVs and stored nodes");

template <int MODE>
__global__ __launch_bounds__(TPB) void km_staged_kernel(MultiArgs a) {
    constexpr int LOGS = 6;
    __shared__ __attribute__((aligned(16))) u32x4 stage[STAGE_VEC * TPB];
    __shared__ __attribute__((aligned(16))) uint32_t cvs[2][S][8];
    __shared__ __attribute__((aligned(16))) uint32_t msg[QUADS][16];
    __shared__ uint32_t last;
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const uint64_t grp = blockIdx.x, N = a.N, n = a.n;
    const uint64_t c0 = grp * S, r = N - c0 < (uint64_t)S ? N - c0 : (uint64_t)S;  // my chunks
    bool ok = true;

    // ---- phase 1 (decode): the header checked, content bytes out
    if (MODE == 1) {
        if (grp == 0 && t == 0 && *reinterpret_cast<const uint64_t *>(a.stream) != n) ok = false;
        const uint64_t lim = a.out ? (a.out_limit < (c0 + r) * 1024 ? a.out_limit : (c0 + r) * 1024) : 0;
        for (uint64_t o = c0 * 1024 + 16 * (uint64_t)t; o < lim; o += 16 * TPB) {
            const uint8_t *p = a.stream + chunk_stream_off(o / 1024, N) + o % 1024;
            const uint64_t left = lim - o;
            if (left >= 16) *glb(reinterpret_cast<u32x4 *>(a.out + o)) = load16_a8(p);
            else store16_partial(a.out + o, load16_partial(p, (uint32_t)left), (uint32_t)left);
        }
    }

    // ---- phase 2a: my range [r0, r1) of the source into LDS (zeros past r1)
    const uint64_t cl = c0 + r - 1;  // my last chunk
    uint64_t r0, r1;
    const uint8_t *src;
    if (MODE == 1) {
        const int sp = parents_at(c0, N);
        r0 = chunk_stream_off(c0, N) - 64 * (uint64_t)(sp < LOGS ? sp : LOGS);  // my left spine's top node
        r1 = chunk_stream_off(cl, N) + (n - 1024 * cl < 1024 ? n - 1024 * cl : 1024);
        src = a.stream;
    } else {
        r0 = c0 * 1024;
        r1 = (c0 + r) * 1024 < a.valid ? (c0 + r) * 1024 : a.valid;
        src = a.src;
    }
    const uint8_t *const sb = reinterpret_cast<const uint8_t *>(stage);
    const uint8_t *al = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(src + r0) & ~uintptr_t(15));
    const uint32_t shift = (uint32_t)(src + r0 - al);  // LDS byte of source byte r0
    {
        const uint8_t *end = src + r1;
        u32x4 v[STAGE_VEC];
#pragma unroll
        for (int j = 0; j < STAGE_VEC; ++j) {
            const uint8_t *p = al + 16 * (uint64_t)(t + TPB * j);
            v[j] = p + 16 <= end ? load16_a8(p) : p < end ? load16_partial(p, (uint32_t)(end - p)) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < STAGE_VEC; ++j) stage[t + TPB * j] = v[j];
    }
    __syncthreads();

    // ---- phase 2b: chunk CVs from LDS, one quad per chunk
    const uint32_t slot = (uint32_t)(reinterpret_cast<uintptr_t>(&msg[g][0]) - reinterpret_cast<uintptr_t>(&msg[0][0]));
    const uint8_t *mbase = reinterpret_cast<const uint8_t *>(&msg[0][0]);
    const small::MsgIdx mi(q, slot);
    const uint32_t iv0 = q == 0 ? IV(0) : q == 1 ? IV(1) : q == 2 ? IV(2) : IV(3);
    const uint32_t iv1 = q == 0 ? IV(4) : q == 1 ? IV(5) : q == 2 ? IV(6) : IV(7);
    if ((uint64_t)g < r) {
        const uint64_t c = c0 + g;
        const uint64_t rem = n - c * 1024;
        const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
        const uint32_t nb = (clen + 63) / 64;  // N >= 2: every chunk holds at least one byte
        const small::MsgIdx mc(q, shift + (uint32_t)((MODE == 1 ? chunk_stream_off(c, N) : c * 1024) - r0));
        uint32_t h0 = iv0, h1 = iv1;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            if ((uint32_t)b < nb) {
                const bool lastb = (uint32_t)b + 1 == nb;
                const uint32_t flags = (b == 0 ? F_CHUNK_START : 0u) | (lastb ? F_CHUNK_END : 0u);
                small::compress4(h0, h1, sb + 64 * b, mc, q, iv0, c, lastb ? clen - 64 * b : 64u, flags);
            }
        }
        cvs[0][g][q] = h0;
        cvs[0][g][4 + q] = h1;
    }
    __syncthreads();

    // ---- phase 3: the group's levels 1 .. 6, one quad per parent
    int cur = 0;
    uint64_t cnt_prev = r;
    for (int level = 1; level <= LOGS && cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        if ((uint64_t)g < cnt) {
            const uint64_t p = g;
            if (2 * p + 1 >= cnt_prev) {  // odd last node: promoted unchanged
                cvs[cur ^ 1][p][q] = cvs[cur][2 * p][q];
                cvs[cur ^ 1][p][4 + q] = cvs[cur][2 * p][4 + q];
            } else {
                const u32x4 mw = *reinterpret_cast<const u32x4 *>(&cvs[cur][2 * p + (q >> 1)][4 * (q & 1)]);
                *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = mw;
                wave_sync();
                uint32_t h0 = iv0, h1 = iv1;
                small::compress4(h0, h1, mbase, mi, q, iv0, 0, 64, F_PARENT);
                wave_sync();
                const uint64_t P = (c0 >> level) + p;
                if (MODE == 0) {
                    node_out(a, P, level, q, mw);
                } else {  // the stored node, staged with my region (4-B aligned words)
                    const uint32_t *s = reinterpret_cast<const uint32_t *>(
                        sb + shift + (parent_stream_off(P << level, level, N) - r0) + 16 * q);
                    ok &= s[0] == mw.x && s[1] == mw.y && s[2] == mw.z && s[3] == mw.w;
                }
                cvs[cur ^ 1][p][q] = h0;
                cvs[cur ^ 1][p][4 + q] = h1;
            }
        }
        __syncthreads();
        cur ^= 1;
        cnt_prev = cnt;
    }
    if (MODE == 1 && !ok) flag_mismatch(a.status, 0);

    // ---- phase 4: publish the group CV; the last workgroup walks the top in
    // the staging area ([2][GMAX][8] CVs, then GMAX * 4 stored node quarters)
    u32x4 *const top = stage;
    km_top<MODE, LOGS>(a, t < 8 ? cvs[cur][0][t] : 0u, reinterpret_cast<uint32_t (*)[GMAX][8]>(top),
                       top + 2 * GMAX * 8 / 4, last, mbase, msg, mi, iv0, iv1);
}

// 16 B of the four parity shards from 16 B at the same position of each data
// shard: the packed parity table ([4][256] dwords in LDS: byte d of entry
// [j][x] = E[4 + d][j] * x), then a 4 x 4 transpose
__device__ __forceinline__ void parity16(const uint32_t *tab, const u32x4 (&v)[4], u32x4 (&p)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t acc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) x ^= tab[j * 256 + ((zf::comp(v[j], d) >> (8 * b)) & 0xFFu)];
            acc[b] = x;
        }
        uint32_t r0, r1, r2, r3;
        zf::transpose4(acc[0], acc[1], acc[2], acc[3], r0, r1, r2, r3);
        if (d == 0) { p[0].x = r0; p[1].x = r1; p[2].x = r2; p[3].x = r3; }
        if (d == 1) { p[0].y = r0; p[1].y = r1; p[2].y = r2; p[3].y = r3; }
        if (d == 2) { p[0].z = r0; p[1].z = r1; p[2].z = r2; p[3].z = r3; }
        if (d == 3) { p[0].w = r0; p[1].w = r1; p[2].w = r2; p[3].w = r3; }
    }
}

// A 4-of-8 zfec encode of one object read from pinned host memory (zero-copy:
// no DMA hop), one 16-B position of every shard per lane (`tiles` > 1:
// positions 4 KiB apart per lane, software-pipelined, the next tile's PCIe
// reads in flight while this tile's results are written; measured slower,
// see parity_tiles).
//   ZC = 0 (km_parity): the data and parity shards into the device stream's
//     chunk slots for KM to hash, the parity shards also into the host image
//     of the stream from t0 on (`tail`, null: none), which is everything of
//     the stream past the data region except its nodes;
//   ZC = 1 (zc_parity, encoding::zfec alone): the 4 parity shards shard-major
//     ([P0|P1|P2|P3], C bytes each) into pinned host memory `out`; the data
//     shards are the zero-padded input, which the host writes itself.
template <int ZC>
__global__ __launch_bounds__(256) void parity_kernel(const uint8_t *in, uint64_t valid, uint64_t C, uint8_t *out,
                                                     uint64_t N, const uint32_t *table, uint8_t *tail, uint64_t t0,
                                                     uint32_t tiles) {
    __shared__ uint32_t tab[4 * 256];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) tab[i] = table[i];
    uint64_t o = 16 * ((uint64_t)blockIdx.x * 256 * tiles + threadIdx.x);
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = o < C ? zf::load16_masked(in, j * C + o, valid) : u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    const uint64_t cols = C / 1024;
    for (uint32_t it = 0; it < tiles; ++it) {
        const uint64_t on = o + 16 * 256;
        u32x4 nv[4];
        const bool more = it + 1 < tiles && on < C;
#pragma unroll
        for (int j = 0; j < 4; ++j) nv[j] = more ? zf::load16_masked(in, j * C + on, valid) : u32x4{0u, 0u, 0u, 0u};
        if (o < C) {
            u32x4 p[4];
            parity16(tab, v, p);
            if (ZC) {
#pragma unroll
                for (int s = 0; s < 4; ++s) *glb(reinterpret_cast<u32x4 *>(out + s * C + o)) = p[s];
            } else {
                const uint64_t u = o / 1024, w = o % 1024;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const uint64_t off = chunk_stream_off(s * cols + u, N) + w;
                    const u32x4 x = s < 4 ? v[s] : p[s - 4];
                    store16_a8<false>(out + off, x);
                    if (s >= 4 && tail) store16_a8<false>(tail + (off - t0), x);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = nv[j];
        o = on;
    }
}

// positions per lane of the parity kernels: CHIP_PARITY_TILES, default 1 (one
// position per lane, the grid covering C).  More tiles pipeline each lane's
// reads and writes but spread the object's PCIe reads over fewer workgroups,
// which costs more than the overlap gains (profiles/NOT_KEPT.md r11zo)
uint32_t parity_tiles(uint64_t C) {
    static const uint32_t env = [] {
        const char *e = std::getenv("CHIP_PARITY_TILES");
        const int v = e ? std::atoi(e) : 1;
        return (uint32_t)(v >= 1 && v <= 64 ? v : 1);
    }();
    const uint64_t tiles_needed = (C / 16 + 255) / 256;  // 4 KiB of every shard per tile
    return (uint32_t)(tiles_needed < env ? (tiles_needed ? tiles_needed : 1) : env);
}

bool enabled() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_KM");
        return !(e && !std::strcmp(e, "0"));
    }();
    return on;
}

// CHIP_KM_STAGE=0: km_kernel everywhere (the A/B against km_staged_kernel)
bool staged_on() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_KM_STAGE");
        return !(e && !std::strcmp(e, "0"));
    }();
    return on;
}

// chunks per workgroup: CHIP_KM_SG (16 / 32 / 64, A/B runs), default 64;
// never so few that the groups overflow the top walk's LDS
int group_chunks(uint64_t N) {
    static const int env = [] {
        const char *e = std::getenv("CHIP_KM_SG");
        const int v = e ? std::atoi(e) : 0;
        return v == 16 || v == 32 || v == 64 ? v : 0;
    }();
    int sg = env ? env : S;
    while (sg < S && (N + sg - 1) / sg > (uint64_t)GMAX) sg *= 2;
    return sg;
}

hipError_t launch(int mode, MultiArgs a, hipStream_t stream) {
    const int sg = group_chunks(a.N);
    const uint64_t G = (a.N + sg - 1) / sg;
    if (a.N <= (uint64_t)S || G > (uint64_t)GMAX) return hipErrorInvalidValue;
    uint32_t *q = nullptr;
    hipError_t e = stream_queue(stream, &q);
    if (e != hipSuccess) return e;
    a.counter = q + QUEUE_KM;
    auto k = mode == 0 ? (sg == 16 ? km_kernel<0, 16> : sg == 32 ? km_kernel<0, 32> : km_kernel<0, 64>)
                       : (sg == 16 ? km_kernel<1, 16> : sg == 32 ? km_kernel<1, 32> : km_kernel<1, 64>);
    // the staged kernel where the chunks come from one contiguous source: the
    // stream to verify (4-B aligned; every region starts >= 72 B into it, so
    // the first 16-B load stays inside) or the content (16-B aligned).  Decode
    // of up to 32 groups keeps km_kernel: with few workgroups its per-block
    // waits overlap the reads better (r11v: 4-8 us faster at 64-256 KiB, even
    // at 1 MiB; the staged rows win from 4 MiB on)
    const uint8_t *from = mode == 1 ? a.stream : a.src;
    if (sg == S && staged_on() && (mode == 1 ? G > 32 : a.n_in == a.N) && from &&
        (reinterpret_cast<uintptr_t>(from) & (mode == 1 ? 3 : 15)) == 0)
        k = mode == 0 ? km_staged_kernel<0> : km_staged_kernel<1>;
    hipLaunchKernelGGL(k, dim3((unsigned)G), dim3(TPB), 0, stream, a);
    return hipGetLastError();
}

}  // namespace multi

bool km_enabled() { return multi::enabled(); }

bool km_ok(uint64_t bao_n, uint64_t count) {
    const uint64_t N = n_chunks(bao_n);
    return multi::enabled() && count == 1 && N > (uint64_t)multi::S && N <= KM_MAX_N;
}

bool single_ok(uint64_t bao_n) {
    if (!multi::enabled() || bao_n == 0) return false;
    const uint64_t N = n_chunks(bao_n);
    return N > (uint64_t)multi::S ? N <= KM_MAX_N : small_ok(bao_n, 1);
}

uint64_t km_scratch_len(uint64_t bao_n) { return 32 * (n_chunks(bao_n) + 15) / 16; }  // any group size

hipError_t km_bao_encode_dev(const uint8_t *d_in, uint64_t n, uint8_t *d_nodes, uint8_t *d_hash, void *d_scratch,
                             hipStream_t stream) {
    multi::MultiArgs a{};
    a.src = d_in; a.nodes = d_nodes;
    a.n = n; a.N = n_chunks(n); a.n_in = a.N; a.valid = n; a.nd = a.N;
    a.hash = d_hash; a.gcv = static_cast<uint8_t *>(d_scratch);
    return multi::launch(0, a, stream);
}

hipError_t km_zfec_bao_dev(const uint8_t *d_in, uint64_t valid, uint64_t C, uint8_t *d_stream, uint8_t *d_nodes,
                           uint8_t *d_tail, uint64_t t0, uint8_t *d_hash, void *d_scratch, hipStream_t stream,
                           hipEvent_t parity_done) {
    if (C == 0 || C % 1024 || !d_stream) return hipErrorInvalidValue;
    const void *tab = nullptr;
    hipError_t e = zfec_parity_table(4, 8, &tab);
    if (e != hipSuccess) return e;
    const uint64_t N = 8 * C / 1024;
    const uint32_t tiles = multi::parity_tiles(C);
    hipLaunchKernelGGL(multi::parity_kernel<0>, dim3((unsigned)((C / 16 + 256 * tiles - 1) / (256 * tiles))), dim3(256),
                       0, stream, d_in, valid, C, d_stream, N, static_cast<const uint32_t *>(tab), d_tail, t0, tiles);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (parity_done && (e = hipEventRecord(parity_done, stream)) != hipSuccess) return e;
    multi::MultiArgs a{};
    a.stream = d_stream; a.nodes = d_nodes; a.tail = d_tail; a.t0 = t0;
    a.n = 8 * C; a.N = N; a.n_in = 0; a.nd = N / 2;
    a.hash = d_hash; a.gcv = static_cast<uint8_t *>(d_scratch);
    return multi::launch(0, a, stream);
}

hipError_t zc_zfec_parity_dev(const uint8_t *d_in, uint64_t valid, uint64_t C, uint8_t *d_par, hipStream_t stream) {
    if (C == 0 || C % 16) return hipErrorInvalidValue;
    const void *tab = nullptr;
    hipError_t e = zfec_parity_table(4, 8, &tab);
    if (e != hipSuccess) return e;
    const uint32_t tiles = multi::parity_tiles(C);
    hipLaunchKernelGGL(multi::parity_kernel<1>, dim3((unsigned)((C / 16 + 256 * tiles - 1) / (256 * tiles))), dim3(256),
                       0, stream, d_in, valid, C, d_par, 0, static_cast<const uint32_t *>(tab), nullptr, 0, tiles);
    return hipGetLastError();
}

hipError_t km_bao_decode_dev(const uint8_t *d_stream, uint64_t n, const uint8_t *d_hash, uint8_t *d_out,
                             uint64_t out_limit, uint32_t *d_status, void *d_scratch, hipStream_t stream) {
    multi::MultiArgs a{};
    a.stream = d_stream; a.out = d_out;
    a.n = n; a.N = n_chunks(n); a.out_limit = d_out ? out_limit : 0;
    a.hash = const_cast<uint8_t *>(d_hash); a.status = d_status;
    a.gcv = static_cast<uint8_t *>(d_scratch);
    return multi::launch(1, a, stream);
}

}  // namespace chip
