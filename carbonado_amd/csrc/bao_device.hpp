// bao_device.hpp — device code of K3/K4/K5 (BLAKE3 chunk CVs, tree levels,
// bao pre-order layout, verify-decode), shared by the product
// (bao_kernels.hip) and tools/bao_tune.hip.  Design notes: bao_kernels.hip.
#pragma once

#include <map>
#include <mutex>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <utility>

#include "chip_internal.hpp"

namespace chip {
namespace bao {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t F_CHUNK_START = 1, F_CHUNK_END = 2, F_PARENT = 4, F_ROOT = 8;
constexpr int K3_WAVES = 4;
constexpr int K3_TPB = 64 * K3_WAVES;
constexpr int ROWW = 36;  // LDS words per staged chunk row: [_, _, carry w30, w31 | 32 data words]
constexpr int ROW0 = 4;   // first data word (16-B aligned; stride 36 keeps b128 reads conflict-free)
// verify-decode reads each chunk pair's level-1 node with the pair's first
// loads (K3 MODE 1, CPL 2); -DBAO_DEC_PREFETCH_DEF=0 builds the old order (A/B)
#ifndef BAO_DEC_PREFETCH_DEF
#define BAO_DEC_PREFETCH_DEF 1
#endif
constexpr bool BAO_DEC_PREFETCH = BAO_DEC_PREFETCH_DEF;

__host__ __device__ constexpr uint32_t IV(int i) {
    return i == 0 ? 0x6A09E667u : i == 1 ? 0xBB67AE85u : i == 2 ? 0x3C6EF372u
         : i == 3 ? 0xA54FF53Au : i == 4 ? 0x510E527Fu : i == 5 ? 0x9B05688Cu
         : i == 6 ? 0x1F83D9ABu : 0x5BE0CD19u;
}

// message schedule: round r reads word SCHED(r, i); round 0 is the identity and
// each round applies the permutation [2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8].
__host__ __device__ constexpr int PERM(int i) {
    constexpr int p[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
    return p[i];
}
__host__ __device__ constexpr int SCHED(int r, int i) { return r == 0 ? i : SCHED(r - 1, PERM(i)); }

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

#define B3G(a, b, c, d, x, y)            \
    do {                                 \
        a = a + b + (x);                 \
        d = rotr(d ^ a, 16);             \
        c = c + d;                       \
        b = rotr(b ^ c, 12);             \
        a = a + b + (y);                 \
        d = rotr(d ^ a, 8);              \
        c = c + d;                       \
        b = rotr(b ^ c, 7);              \
    } while (0)

// Four independent G's issued step by step, each step applied to all four
// before the next (inline asm keeps the order; the compiler interleaves
// other work around it).  The same instructions as B3G in a fixed order:
// the compiler's own order ran the compression loop at 5.69e10 per second
// at 8 waves/SIMD, this one at 6.13e10 (+7.6 %; +1.5 % at 2 waves/SIMD;
// tools/valu_probe.hip VAR 3, profiles/r6q_valu_probe.txt).
#ifndef B3_GROUPED_DEF
#define B3_GROUPED_DEF 1
#endif
constexpr bool B3_GROUPED = B3_GROUPED_DEF;
#define B3_ADD3(d, x, y) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(d) : "v"(x), "v"(y))
#define B3_XOR(d, x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(x))
#define B3_ROT(d, n) asm volatile("v_alignbit_b32 %0, %0, %0, " #n : "+v"(d))
#define B3_ADD(d, x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(x))
// One asm statement per four G's (B3_ONEASM 1) with an `s_nop 0` after each
// group of four VOP2 ops (the xors and adds), none after the VOP3 groups
// (add3, alignbit).  With one statement per instruction the hazard
// recognizer, blind inside asm, puts an `s_nop 0` before every group that
// reads the previous group's results.  Measured (tools/valu_probe.hip VAR 3/4/6/7,
// profiles/r7c, r7d): without any nop the compression loop runs 6 % slower at 8
// waves/SIMD (5.73 vs 6.11e10/s) — a group issued right behind four
// full-rate VOP2 producers stalls on them — and with nops after the VOP2
// groups only it runs as fast at 8 waves and ~1 % faster at 2-3 waves
// (5.60/5.76 vs 5.55/5.69e10/s), the occupancies of K13 and verify-decode.
#ifndef B3_ONEASM_DEF
#define B3_ONEASM_DEF 1
#endif
// B3_PK16 1: the rotate by 16 of each G as v_pk_add_u16 with swapped halves
// (x.hi + 0 | (x.lo + 0) << 16) instead of v_alignbit_b32 (tools/valu_probe
// "pk", VAR 13/14); the other rotations stay alignbit.
#ifndef B3_PK16_DEF
#define B3_PK16_DEF 0
#endif
#if B3_PK16_DEF
#define B3_ROT16_4                                                                                     \
    "v_pk_add_u16 %12, %12, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\tv_pk_add_u16 %13, %13, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\t" \
    "v_pk_add_u16 %14, %14, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\tv_pk_add_u16 %15, %15, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\t"
#else
#define B3_ROT16_4                                                                                     \
    "v_alignbit_b32 %12, %12, %12, 16\n\tv_alignbit_b32 %13, %13, %13, 16\n\t"                          \
    "v_alignbit_b32 %14, %14, %14, 16\n\tv_alignbit_b32 %15, %15, %15, 16\n\t"
#endif
__device__ __forceinline__ void b3_g4(uint32_t &a0, uint32_t &b0, uint32_t &c0, uint32_t &d0, uint32_t &a1,
                                      uint32_t &b1, uint32_t &c1, uint32_t &d1, uint32_t &a2, uint32_t &b2,
                                      uint32_t &c2, uint32_t &d2, uint32_t &a3, uint32_t &b3, uint32_t &c3,
                                      uint32_t &d3, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t x2,
                                      uint32_t y2, uint32_t x3, uint32_t y3) {
    if constexpr (B3_ONEASM_DEF) {
        // operands: a0..a3 = 0..3, b = 4..7, c = 8..11, d = 12..15, x = 16..19, y = 20..23
        asm volatile(
            "v_add3_u32 %0, %0, %4, %16\n\tv_add3_u32 %1, %1, %5, %17\n\t"
            "v_add3_u32 %2, %2, %6, %18\n\tv_add3_u32 %3, %3, %7, %19\n\t"
            "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\t"
            "s_nop 0\n\t"
            B3_ROT16_4
            "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\t"
            "s_nop 0\n\t"
            "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\t"
            "s_nop 0\n\t"
            "v_alignbit_b32 %4, %4, %4, 12\n\tv_alignbit_b32 %5, %5, %5, 12\n\t"
            "v_alignbit_b32 %6, %6, %6, 12\n\tv_alignbit_b32 %7, %7, %7, 12\n\t"
            "v_add3_u32 %0, %0, %4, %20\n\tv_add3_u32 %1, %1, %5, %21\n\t"
            "v_add3_u32 %2, %2, %6, %22\n\tv_add3_u32 %3, %3, %7, %23\n\t"
            "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\t"
            "s_nop 0\n\t"
            "v_alignbit_b32 %12, %12, %12, 8\n\tv_alignbit_b32 %13, %13, %13, 8\n\t"
            "v_alignbit_b32 %14, %14, %14, 8\n\tv_alignbit_b32 %15, %15, %15, 8\n\t"
            "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\t"
            "s_nop 0\n\t"
            "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\t"
            "s_nop 0\n\t"
            "v_alignbit_b32 %4, %4, %4, 7\n\tv_alignbit_b32 %5, %5, %5, 7\n\t"
            "v_alignbit_b32 %6, %6, %6, 7\n\tv_alignbit_b32 %7, %7, %7, 7"
            : "+&v"(a0), "+&v"(a1), "+&v"(a2), "+&v"(a3), "+&v"(b0), "+&v"(b1), "+&v"(b2), "+&v"(b3),
              "+&v"(c0), "+&v"(c1), "+&v"(c2), "+&v"(c3), "+&v"(d0), "+&v"(d1), "+&v"(d2), "+&v"(d3)
            : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(y0), "v"(y1), "v"(y2), "v"(y3));
        return;
    }
    B3_ADD3(a0, b0, x0); B3_ADD3(a1, b1, x1); B3_ADD3(a2, b2, x2); B3_ADD3(a3, b3, x3);
    B3_XOR(d0, a0); B3_XOR(d1, a1); B3_XOR(d2, a2); B3_XOR(d3, a3);
    B3_ROT(d0, 16); B3_ROT(d1, 16); B3_ROT(d2, 16); B3_ROT(d3, 16);
    B3_ADD(c0, d0); B3_ADD(c1, d1); B3_ADD(c2, d2); B3_ADD(c3, d3);
    B3_XOR(b0, c0); B3_XOR(b1, c1); B3_XOR(b2, c2); B3_XOR(b3, c3);
    B3_ROT(b0, 12); B3_ROT(b1, 12); B3_ROT(b2, 12); B3_ROT(b3, 12);
    B3_ADD3(a0, b0, y0); B3_ADD3(a1, b1, y1); B3_ADD3(a2, b2, y2); B3_ADD3(a3, b3, y3);
    B3_XOR(d0, a0); B3_XOR(d1, a1); B3_XOR(d2, a2); B3_XOR(d3, a3);
    B3_ROT(d0, 8); B3_ROT(d1, 8); B3_ROT(d2, 8); B3_ROT(d3, 8);
    B3_ADD(c0, d0); B3_ADD(c1, d1); B3_ADD(c2, d2); B3_ADD(c3, d3);
    B3_XOR(b0, c0); B3_XOR(b1, c1); B3_XOR(b2, c2); B3_XOR(b3, c3);
    B3_ROT(b0, 7); B3_ROT(b1, 7); B3_ROT(b2, 7); B3_ROT(b3, 7);
}

template <int R>
__device__ __forceinline__ void b3_round(uint32_t (&v)[16], const uint32_t (&m)[16]) {
    if constexpr (B3_GROUPED) {
        b3_g4(v[0], v[4], v[8], v[12], v[1], v[5], v[9], v[13], v[2], v[6], v[10], v[14], v[3], v[7], v[11], v[15],
              m[SCHED(R, 0)], m[SCHED(R, 1)], m[SCHED(R, 2)], m[SCHED(R, 3)], m[SCHED(R, 4)], m[SCHED(R, 5)],
              m[SCHED(R, 6)], m[SCHED(R, 7)]);
        b3_g4(v[0], v[5], v[10], v[15], v[1], v[6], v[11], v[12], v[2], v[7], v[8], v[13], v[3], v[4], v[9], v[14],
              m[SCHED(R, 8)], m[SCHED(R, 9)], m[SCHED(R, 10)], m[SCHED(R, 11)], m[SCHED(R, 12)], m[SCHED(R, 13)],
              m[SCHED(R, 14)], m[SCHED(R, 15)]);
        return;
    }
    B3G(v[0], v[4], v[8], v[12], m[SCHED(R, 0)], m[SCHED(R, 1)]);
    B3G(v[1], v[5], v[9], v[13], m[SCHED(R, 2)], m[SCHED(R, 3)]);
    B3G(v[2], v[6], v[10], v[14], m[SCHED(R, 4)], m[SCHED(R, 5)]);
    B3G(v[3], v[7], v[11], v[15], m[SCHED(R, 6)], m[SCHED(R, 7)]);
    B3G(v[0], v[5], v[10], v[15], m[SCHED(R, 8)], m[SCHED(R, 9)]);
    B3G(v[1], v[6], v[11], v[12], m[SCHED(R, 10)], m[SCHED(R, 11)]);
    B3G(v[2], v[7], v[8], v[13], m[SCHED(R, 12)], m[SCHED(R, 13)]);
    B3G(v[3], v[4], v[9], v[14], m[SCHED(R, 14)], m[SCHED(R, 15)]);
}

// h <- first 8 output words of compress(h, m, counter, blen, flags)
__device__ __forceinline__ void b3_compress(uint32_t (&h)[8], const uint32_t (&m)[16], uint64_t ctr,
                                            uint32_t blen, uint32_t flags) {
    uint32_t v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7],
                      IV(0), IV(1), IV(2), IV(3),
                      (uint32_t)ctr, (uint32_t)(ctr >> 32), blen, flags};
    b3_round<0>(v, m); b3_round<1>(v, m); b3_round<2>(v, m); b3_round<3>(v, m);
    b3_round<4>(v, m); b3_round<5>(v, m); b3_round<6>(v, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = v[i] ^ v[i + 8];
}

// The same with f(r) called after round r (fused_tune: instructions placed
// between the rounds, e.g. stores spread over a compression).
template <class F>
__device__ __forceinline__ void b3_compress_cb(uint32_t (&h)[8], const uint32_t (&m)[16], uint64_t ctr,
                                               uint32_t blen, uint32_t flags, F &&f) {
    uint32_t v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7],
                      IV(0), IV(1), IV(2), IV(3),
                      (uint32_t)ctr, (uint32_t)(ctr >> 32), blen, flags};
    b3_round<0>(v, m); f(0); b3_round<1>(v, m); f(1); b3_round<2>(v, m); f(2); b3_round<3>(v, m); f(3);
    b3_round<4>(v, m); f(4); b3_round<5>(v, m); f(5); b3_round<6>(v, m); f(6);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = v[i] ^ v[i + 8];
}

__device__ __forceinline__ void b3_parent(const uint32_t (&l)[8], const uint32_t (&r)[8], bool root,
                                          uint32_t (&out)[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) { m[i] = l[i]; m[8 + i] = r[i]; out[i] = IV(i); }
    b3_compress(out, m, 0, 64, F_PARENT | (root ? F_ROOT : 0));
}

__host__ __device__ __forceinline__ int ceil_log2(uint64_t x) {  // x >= 1
#if defined(__HIP_DEVICE_COMPILE__)
    return x <= 1 ? 0 : 64 - __clzll((long long)(x - 1));
#else
    return x <= 1 ? 0 : 64 - __builtin_clzll(x - 1);
#endif
}

__host__ __device__ __forceinline__ int ctz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ffsll((long long)x) - 1;
#else
    return __builtin_ctzll(x);
#endif
}

// c(s): parents whose leftmost chunk is s
__host__ __device__ __forceinline__ int parents_at(uint64_t s, uint64_t N) {
    const int cl = ceil_log2(N - s);
    if (s == 0) return cl;
    const int tz = ctz64(s);
    return tz < cl ? tz : cl;
}

// P(s): parents whose leftmost chunk is < s
__host__ __device__ __forceinline__ uint64_t parents_before(uint64_t s, uint64_t N) {
    uint64_t total = 0, cnt = N;
    for (int L = 1; cnt > 1; ++L) {
        const uint64_t np = cnt / 2;
        const uint64_t before = (s + (1ull << L) - 1) >> L;
        total += before < np ? before : np;
        cnt = (cnt + 1) / 2;
    }
    return total;
}

__host__ __device__ __forceinline__ uint64_t chunk_stream_off(uint64_t i, uint64_t N) {
    return 8 + 1024 * i + 64 * (parents_before(i, N) + parents_at(i, N));
}

__host__ __device__ __forceinline__ uint64_t parent_stream_off(uint64_t s, int level, uint64_t N) {
    return 8 + 1024 * s + 64 * (parents_before(s, N) + parents_at(s, N) - level);
}

__device__ __forceinline__ u32x4 load16_partial(const uint8_t *p, uint32_t valid) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((uint32_t)i < valid) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    u32x4 r = {w[0], w[1], w[2], w[3]};
    return r;
}

__device__ __forceinline__ void store16_partial(uint8_t *p, u32x4 v, uint32_t valid) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if ((uint32_t)i < valid) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// 16 bytes at an 8-byte-aligned address
typedef uint32_t u32x4_a8 __attribute__((ext_vector_type(4), aligned(8)));
__device__ __forceinline__ u32x4 load16_a8(const uint8_t *p) {  // one dwordx4 load (gfx950: unaligned OK)
    const u32x4_a8 v = *reinterpret_cast<const u32x4_a8 *>(p);
    return u32x4{v.x, v.y, v.z, v.w};
}



// Nearest real parent above the node (level lv, leftmost chunk sx): the lowest
// level lp > lv whose node containing sx has two children.  Returns 0 when the
// node is the root.  The node is that parent's left child iff sx is the
// parent's leftmost chunk (a promoted node keeps its leftmost chunk).
__host__ __device__ __forceinline__ int nearest_parent(uint64_t sx, int lv, uint64_t N, uint64_t *sp) {
    for (int lp = lv + 1; lp < 64; ++lp) {
        const uint64_t s0 = (sx >> lp) << lp;
        if (s0 + (1ull << (lp - 1)) < N) { *sp = s0; return lp; }
        if (s0 == 0 && (1ull << lp) >= N) return 0;
    }
    return 0;
}

// bao's top-down check of one node, restated per node: does the CV `cv` of
// the node (level lv, leftmost chunk sx) equal the copy stored in its parent?
__device__ __forceinline__ bool stored_slot_matches(const uint8_t *stream, uint64_t sx, int lv, uint64_t N,
                                                    const uint32_t (&cv)[8]) {
    uint64_t sp = 0;
    const int lp = nearest_parent(sx, lv, N, &sp);
    const uint8_t *slot = stream + parent_stream_off(sp, lp, N) + (sx == sp ? 0 : 32);
    bool ok = true;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const u32x2 x = reinterpret_cast<const u32x2 *>(slot)[w];
        ok &= x.x == cv[2 * w] && x.y == cv[2 * w + 1];
    }
    return ok;
}

struct ChunkArgs {
    const uint8_t *in;
    uint8_t *out;          // encode: stream (may be null = hash only); decode: content
    uint64_t in_stride, out_stride;
    uint64_t n, N, count;
    uint8_t *cv;           // level-log2(CPL) node CVs: [count][cv_stride] x 32 B
    uint64_t cv_stride;
    uint8_t *hash;         // encode: root hash out (when the root is formed here); decode: expected
    uint32_t *status;      // decode only
    uint64_t out_limit = ~0ull;  // decode: content bytes at or past it are verified, not written
    uint32_t *queue = nullptr;   // DQ: [0] next wave task, [32] waves done
};

__device__ __forceinline__ void wave_sync() {
    // Every LDS row a wave writes is read only by lanes of the same wave, and
    // a wave's DS instructions execute in order: a compiler-level fence is all
    // that is needed to keep the reads after the writes (no s_barrier).
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// A generic pointer as a global-memory one.  Stores through a pointer whose
// address space the compiler cannot trace (one passed through __shfl, or
// picked from a per-lane array) compile to flat_store; flat instructions
// count in LGKM_CNT as well as VM_CNT and complete out of order, so the next
// LDS read's s_waitcnt lgkmcnt(0) would wait for every such store in flight.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *glb(T *p) {
    return (__attribute__((address_space(1))) T *)p;
}

template <bool NT>
__device__ __forceinline__ void store8(uint8_t *p, u32x2 v) {
    if (NT) __builtin_nontemporal_store(v, glb(reinterpret_cast<u32x2 *>(p)));
    else *glb(reinterpret_cast<u32x2 *>(p)) = v;
}

template <bool NT>
__device__ __forceinline__ void store16_a8(uint8_t *p, u32x4 v) {
    store8<NT>(p, u32x2{v.x, v.y});
    store8<NT>(p + 8, u32x2{v.z, v.w});
}

// encode: write parent node (l || r) at `node`; decode: compare with the stored node
template <int MODE, bool NT>
__device__ __forceinline__ bool node_io(uint8_t *node, const uint32_t (&l)[8], const uint32_t (&r)[8]) {
    if (MODE == 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            store8<NT>(node + 8 * w, u32x2{l[2 * w], l[2 * w + 1]});
            store8<NT>(node + 32 + 8 * w, u32x2{r[2 * w], r[2 * w + 1]});
        }
        return true;
    }
    bool ok = true;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const u32x2 x = reinterpret_cast<const u32x2 *>(node)[w];
        const u32x2 y = reinterpret_cast<const u32x2 *>(node + 32)[w];
        ok &= x.x == l[2 * w] && x.y == l[2 * w + 1] && y.x == r[2 * w] && y.y == r[2 * w + 1];
    }
    return ok;
}

__device__ __forceinline__ void flag_mismatch(uint32_t *status, uint64_t obj) {
    __hip_atomic_store(status + obj, (uint32_t)CHIP_ERR_BAO_HASH_MISMATCH, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__device__ __forceinline__ void root_io(const ChunkArgs &a, uint64_t obj, const uint32_t (&h)[8]) {
    u32x4 *hp = reinterpret_cast<u32x4 *>(a.hash + obj * 32);
    if (MODE == 0) {
        hp[0] = u32x4{h[0], h[1], h[2], h[3]};
        hp[1] = u32x4{h[4], h[5], h[6], h[7]};
    } else {
        const u32x4 e0 = hp[0], e1 = hp[1];
        const bool ok = e0.x == h[0] && e0.y == h[1] && e0.z == h[2] && e0.w == h[3] && e1.x == h[4] &&
                        e1.y == h[5] && e1.z == h[6] && e1.w == h[7];
        if (!ok) flag_mismatch(a.status, obj);
    }
}

__host__ __device__ constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

// K3.  MODE 0 = encode (in = content, out = stream), MODE 1 = verify-decode
// (in = stream, out = content), MODE 2 = per-node check (slices, scrub),
// MODE 3 = encode in place (in = out = a stream whose chunk slots already
// hold the content, e.g. written there by the zfec kernel: only the header,
// the parents and the hash are produced).  Lane = CPL consecutive chunks [lb, lb+CPL),
// hashed one after another, their first log2(CPL) tree levels folded in
// registers (BLAKE3 CV stack); a wave = 64*CPL consecutive chunks.  Each of
// the 8*CPL steps stages 128 B of the current chunk of every lane in the
// wave through LDS (coalesced 16-B loads, 8 lanes = one 128-B line), with the
// next step's loads prefetched into registers while the lane compresses.
// SP (stream path, MODE 0): 0 = aligned pieces re-read from the LDS rows;
// 1 = pieces built in registers from the loaded data (DPP neighbour exchange);
// 2 = diagnostic for tools/bao_tune only (128-B aligned bases, wrong layout);
// 3 = rows hold two steps (ping-pong) and every step stores one whole aligned
//     128-B line of the stream per chunk (plus the head at step 0 and the
//     tail at step 7), so no line is written in two halves.
// SE 2 / 3: diagnostics for tools/bao_tune (LDS reads without the stores /
// stores without the LDS reads; wrong output).  SE 6 (MODE 1, diagnostic,
// wrong output): every chunk read from its slot rounded down to a 128-B
// line, so no memory line is shared by two owners and fetched twice, and no
// level-1 node is read: verify-decode's time without its duplicated
// border-line fetches, at the product's occupancy.
// SU: unroll of the SP 3 store loop; SE: issue the SP 3 stores before (1) or
// after (0) the next step's prefetch loads.
// XG 1: XCD-grouped block order (block b runs logical block (b % 8) * (B/8) + b/8,
// so each XCD sweeps one contiguous eighth of the batch; B % 8 == 0 only).
// DQ: persistent grid, wave tasks from the run queue a.queue (zero at launch).
// This is the kernel body; ChunkKernel below names the kernel launched for a
// configuration.
template <int MODE, int CPL, bool NTS, int SP = 0, int SU = 1, int SE = 0, int XG = 0, bool DQ = false>
__device__ __forceinline__ void bao_chunk_body(const ChunkArgs &a) {
    constexpr int LOG = ilog2(CPL);
    constexpr int NSTEP = 8 * CPL;
    // SP 3: [pad 4 | step-parity-0 data 32 | step-parity-1 data 32] words per row
    // (68/4 = 17 is odd, so the lane-per-row ds_read_b128 stays conflict-free)
    constexpr int RW = SP == 3 ? 68 : ROWW;
    __shared__ __attribute__((aligned(16))) uint32_t stage[K3_WAVES][64 * RW];
    auto dofs = [](int step) { return ROW0 + (SP == 3 ? (step & 1) * 32 : 0); };
    __shared__ uint64_t soff[2][K3_WAVES][64];  // stream offset of each lane's current chunk (by parity)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint64_t span = 64ull * CPL;
    const uint64_t tpo = (a.N + span - 1) / span;
    uint64_t blk = blockIdx.x;
    if (!DQ && XG && (gridDim.x & 7) == 0) blk = (blk & 7) * (gridDim.x >> 3) + (blk >> 3);
    // DQ: wave tasks from a run queue (one atomic per task, lane 0; vector
    // memory), persistent grid: the slower XCDs take fewer tasks.  Otherwise
    // one task per wave of the grid.
    const uint64_t ntasks = a.count * tpo;
    auto grab = [&]() -> uint64_t {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(a.queue, 1u);
        return (uint64_t)__builtin_amdgcn_readfirstlane(b);
    };
    for (uint64_t wt = DQ ? grab() : blk * K3_WAVES + wave;; wt = grab()) {
        if (DQ && wt >= ntasks) break;
        const bool wave_on = wt < a.count * tpo;
        const uint64_t obj = wave_on ? wt / tpo : 0;
        const uint64_t c0 = wave_on ? (wt - obj * tpo) * span : 0;
        const uint64_t lb = c0 + (uint64_t)lane * CPL;  // my first chunk
        const uint64_t nmine = (wave_on && lb < a.N) ? ((a.N - lb) < (uint64_t)CPL ? (a.N - lb) : (uint64_t)CPL) : 0;
        const uint8_t *ib = a.in + obj * a.in_stride;
        uint8_t *ob = a.out ? a.out + obj * a.out_stride : nullptr;
        uint32_t *st = stage[wave];

        uint64_t my_off = nmine ? chunk_stream_off(lb, a.N) : 0;  // stream offset of my current chunk
        soff[0][wave][lane] = my_off;
        if ((MODE == 0 || MODE == 3) && ob && wave_on && c0 == 0 && lane == 0)  // u64 LE content-length header
            *reinterpret_cast<uint64_t *>(ob) = a.n;
        if ((MODE == 1 || MODE == 2) && wave_on && c0 == 0 && lane == 0 && *reinterpret_cast<const uint64_t *>(ib) != a.n && a.status)
            flag_mismatch(a.status, obj);  // header disagrees with the batch's content length
        wave_sync();

        // Fast path: every chunk of this wave is a full 1 KiB chunk of the object
        // (all but the last wave of an object), so no per-load bounds logic: the
        // content address is a wave-uniform base + a per-lane constant + t*8*CPL KiB,
        // and stream-mode chunk offsets are fetched from LDS once per chunk round.
        const bool full_wave = wave_on && c0 + span <= a.n / 1024;
        const uint32_t lane_off = (uint32_t)((lane & 7) * 16 + (lane >> 3) * CPL * 1024);
        uint64_t soff_t[8];  // MODE != 0: stream offset of chunk t*8 + lane/8 of the current round
        // loader view: step g covers chunk j = g/8 of every lane, bytes [128*(g%8), +128)
        auto load_step = [&](int g, u32x4 (&v)[8]) {
            const int j = g >> 3, s = g & 7;
            if (full_wave) {
                if (MODE == 0) {
                    const uint8_t *b = ib + (c0 + j) * 1024 + s * 128 + lane_off;
    #pragma unroll
                    for (int t = 0; t < 8; ++t)
                        v[t] = *reinterpret_cast<const u32x4 *>(b + (uint64_t)t * 8 * CPL * 1024);
                } else {
                    if (s == 0) {
    #pragma unroll
                        for (int t = 0; t < 8; ++t) soff_t[t] = soff[j & 1][wave][t * 8 + (lane >> 3)];
                    }
                    const uint8_t *b = ib + s * 128 + (lane & 7) * 16;
                    if constexpr (SE == 6) {  // diagnostic: each chunk read from its slot rounded down to 128 B
    #pragma unroll
                        for (int t = 0; t < 8; ++t)
                            v[t] = *reinterpret_cast<const u32x4 *>(b + (soff_t[t] & ~(uint64_t)127));
                        return;
                    }
    #pragma unroll
                    for (int t = 0; t < 8; ++t) v[t] = load16_a8(b + soff_t[t]);
                }
                return;
            }
    #pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int cc = t * 8 + (lane >> 3);
                const uint64_t ci = c0 + (uint64_t)cc * CPL + j;
                const uint32_t byte = (uint32_t)(s * 128 + (lane & 7) * 16);
                v[t] = u32x4{0u, 0u, 0u, 0u};
                if (wave_on && ci < a.N) {
                    const uint64_t rem = a.n - ci * 1024;
                    const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
                    if (byte < clen) {
                        const uint32_t valid = clen - byte;
                        const uint8_t *src = MODE == 0 ? ib + ci * 1024 + byte : ib + soff[j & 1][wave][cc] + byte;  // 1, 2: stream
                        if (valid >= 16) v[t] = MODE == 0 ? *reinterpret_cast<const u32x4 *>(src) : load16_a8(src);
                        else v[t] = load16_partial(src, valid);
                    }
                }
            }
        };
        // decode: content is 16-B aligned, store straight from the loaded registers
        auto content_step = [&](int g, const u32x4 (&v)[8]) {
            const int j = g >> 3, s = g & 7;
            if (full_wave && (c0 + span) * 1024 <= a.out_limit) {  // the loads' fast-path address pattern, in the content buffer
                uint8_t *b = ob + (c0 + j) * 1024 + s * 128 + lane_off;
    #pragma unroll
                for (int t = 0; t < 8; ++t) {
                    u32x4 *q = reinterpret_cast<u32x4 *>(b + (uint64_t)t * 8 * CPL * 1024);
                    if (NTS) __builtin_nontemporal_store(v[t], q);
                    else *q = v[t];
                }
                return;
            }
    #pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int cc = t * 8 + (lane >> 3);
                const uint64_t ci = c0 + (uint64_t)cc * CPL + j;
                const uint32_t byte = (uint32_t)(s * 128 + (lane & 7) * 16);
                if (!(wave_on && ci < a.N) || ci * 1024 >= a.out_limit) continue;
                const uint64_t rem = (a.n < a.out_limit ? a.n : a.out_limit) - ci * 1024;
                const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
                if (byte >= clen) continue;
                const uint32_t valid = clen - byte;
                uint8_t *dst = ob + ci * 1024 + byte;
                if (valid >= 16) {
                    if (NTS) __builtin_nontemporal_store(v[t], reinterpret_cast<u32x4 *>(dst));
                    else *reinterpret_cast<u32x4 *>(dst) = v[t];
                } else {
                    store16_partial(dst, v[t], valid);
                }
            }
        };
        // encode: chunks sit at stream offsets = 8 (mod 16), so lane g of a chunk's
        // 8-lane group emits the 16-B ALIGNED piece k = 8s+g covering chunk bytes
        // [16k-8, 16k+8): the previous step's last 8 bytes live in the row's carry
        // words, so every full piece is one aligned dwordx4 store read from LDS.
        // Chunk head (k = 0) and tail (k = 64) are 8-byte halves.
        // SP 0: stores of the issuing wave's own rows (wv = wave)
        auto stream_step = [&](int wv, int g) {
            const int j = g >> 3, s = g & 7, gl = lane & 7;
            const uint64_t wt_w = blk * K3_WAVES + wv;
            const bool on_w = wt_w < a.count * tpo;
            const uint64_t obj_w = on_w ? wt_w / tpo : 0;
            const uint64_t c0_w = on_w ? (wt_w - obj_w * tpo) * span : 0;
            uint8_t *ob_w = a.out + obj_w * a.out_stride;
            const uint32_t *st_w = stage[wv];
    #pragma unroll 1
            for (int t = 0; t < 8; ++t) {
                const int cc = t * 8 + (lane >> 3);
                const uint64_t ci = c0_w + (uint64_t)cc * CPL + j;
                if (!(on_w && ci < a.N)) continue;
                const uint64_t rem = a.n - ci * 1024;
                const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
                uint8_t *base = ob_w + soff[j & 1][wv][cc];
                const uint32_t *w = st_w + cc * RW + 2 + 4 * gl;  // carry/previous half, then this piece
                const int lo = 16 * (8 * s + gl) - 8;             // chunk byte of the piece's first half
                if (clen == 1024) {
                    if (lo >= 0) {
                        const u32x2 x = *reinterpret_cast<const u32x2 *>(w);
                        const u32x2 y = *reinterpret_cast<const u32x2 *>(w + 2);
                        const u32x4 v = {x.x, x.y, y.x, y.y};
                        if (NTS) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(base + lo));
                        else *reinterpret_cast<u32x4 *>(base + lo) = v;
                    } else {  // head: chunk bytes [0, 8)
                        store8<NTS>(base, *reinterpret_cast<const u32x2 *>(w + 2));
                    }
                    if (s == 7 && gl == 7)  // tail: chunk bytes [1016, 1024)
                        store8<NTS>(base + 1016, *reinterpret_cast<const u32x2 *>(w + 4));
                } else {  // short last chunk of the object: byte stores
                    for (int q = 0; q < 16; ++q) {
                        const int cb = lo + q;
                        if (cb >= 0 && (uint32_t)cb < clen)
                            base[cb] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
                    }
                    if (s == 7 && gl == 7)
                        for (int q = 0; q < 8; ++q)
                            if (1016u + q < clen) base[1016 + q] = (uint8_t)(w[4 + (q >> 2)] >> (8 * (q & 3)));
                }
            }
        };

        // encode, SP 1: straight from the loaded registers.  Lane g of a chunk's
        // 8-lane group holds chunk bytes [128s+16g, +16) at stream offset 8 (mod 16);
        // it stores the ALIGNED 16 B [128s+16g+8, +16) = its upper half + the next
        // lane's lower half (DPP row_shl:1), lane 0 adds the 8-B head of the step
        // and lane 7 the 8-B tail, so a step needs no bytes of its neighbours.
        auto stream_regs = [&](int g, const u32x4 (&v)[8]) {
            const int j = g >> 3, s = g & 7, gl = lane & 7;
            uint64_t bo[8];
    #pragma unroll
            for (int t = 0; t < 8; ++t) bo[t] = soff[j & 1][wave][t * 8 + (lane >> 3)];
    #pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t nx = __builtin_amdgcn_update_dpp(0u, v[t].x, 0x101, 0xF, 0xF, false);
                const uint32_t ny = __builtin_amdgcn_update_dpp(0u, v[t].y, 0x101, 0xF, 0xF, false);
                const int cc = t * 8 + (lane >> 3);
                const uint64_t ci = c0 + (uint64_t)cc * CPL + j;
                if (!(wave_on && ci < a.N)) continue;
                const uint64_t rem = a.n - ci * 1024;
                const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
                if (SP == 2) {
                    uint8_t *q = ob + (bo[t] & ~127ull) + 128 * s + 16 * gl;
                    if (clen == 1024) *reinterpret_cast<u32x4 *>(q) = v[t];
                    continue;
                }
                uint8_t *p = ob + bo[t] + 128 * s + 16 * gl;
                if (clen == 1024) {
                    if (gl < 7) {
                        const u32x4 o = {v[t].z, v[t].w, nx, ny};
                        if (NTS) __builtin_nontemporal_store(o, reinterpret_cast<u32x4 *>(p + 8));
                        else *reinterpret_cast<u32x4 *>(p + 8) = o;
                    }
                    if (gl == 0 || gl == 7)
                        store8<NTS>(gl == 0 ? p : p + 8, gl == 0 ? u32x2{v[t].x, v[t].y} : u32x2{v[t].z, v[t].w});
                } else {  // short last chunk of the object
                    const uint32_t cb = 128u * s + 16u * gl;
                    if (cb < clen) store16_partial(p, v[t], clen - cb);
                }
            }
        };

        // encode, SP 3: chunk bytes x live in the row at word dofs(x >> 7) + (x & 127) / 4.
        // The stream lines (128-B aligned in stream space) inside a chunk start at
        // chunk byte d + 128 t, d = (-base) mod 128; at step s the line ending at
        // d + 128 s is complete (its first part is in the other half of the row).
        uint32_t diag = 0;  // SE 2 diagnostic sink
        uint8_t *lsp[8];  // SP 3 fast path: stream address and line phase of chunk t*8 + lane/8, per round
        uint32_t ldd[8];
        auto stream_lines = [&](int g) {
            const int j = g >> 3, s = g & 7, gl = lane & 7;
            // 8 B at chunk byte x (8-aligned): the two step halves after the 16-B
            // pad are one 256-B ring (SP 3's only layout), byte x at pad + x mod 256
            auto piece = [&](const uint32_t *row, uint32_t x) -> u32x2 {
                static_assert(SP != 3 || RW == 68, "ring layout");
                return *reinterpret_cast<const u32x2 *>(reinterpret_cast<const uint8_t *>(row) + 4 * ROW0 + (x & 255u));
            };
            if (full_wave) {  // all chunks full: per-chunk values computed once per round
                if (s == 0) {
    #pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        lsp[t] = ob + soff[j & 1][wave][t * 8 + (lane >> 3)];
                        ldd[t] = (uint32_t)(-(uintptr_t)lsp[t]) & 127u;
                    }
                }
    #pragma unroll SU
                for (int t = 0; t < 8; ++t) {
                    uint8_t *sp = lsp[t];
                    const uint32_t d = ldd[t];
                    const uint32_t *row = st + (t * 8 + (lane >> 3)) * RW;
                    if (s >= 1) {  // the whole line [d + 128(s-1), d + 128 s)
                        const uint32_t x = d + 128u * (s - 1) + 16u * gl;
                        if constexpr (SE == 3) {  // diagnostic (tools/bao_tune): the stores without the LDS reads
                            *reinterpret_cast<u32x4 *>(sp + x) = u32x4{x, d, x, d};
                            continue;
                        }
                        if constexpr (SE == 4) {  // diagnostic: as 3, every wave rewriting the same 8 KiB (L2 hits)
                            *reinterpret_cast<u32x4 *>(ob + t * 1024 + lane * 16) = u32x4{x, d, x, d};
                            continue;
                        }
                        if constexpr (SE == 5) {  // diagnostic: as 3, half the stores
                            if (t & 1) continue;
                            *reinterpret_cast<u32x4 *>(sp + x) = u32x4{x, d, x, d};
                            continue;
                        }
                        const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                        const u32x4 v = {lo.x, lo.y, hi.x, hi.y};
                        if constexpr (SE == 2) {  // diagnostic: the LDS reads without the stores
                            diag ^= v.x ^ v.w;
                            continue;
                        }
                        if (NTS) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(sp + x));
                        else *reinterpret_cast<u32x4 *>(sp + x) = v;
                    } else {  // head [0, d)
                        const uint32_t h = d & 8u;
                        if (h && gl == 0) store8<NTS>(sp, piece(row, 0));
                        const uint32_t x = 16u * gl + h;
                        if (x + 16 <= d) {
                            const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                            *reinterpret_cast<u32x4 *>(sp + x) = u32x4{lo.x, lo.y, hi.x, hi.y};
                        }
                    }
                    if (s == 7) {  // tail [896 + d, 1024)
                        const uint32_t x = 896u + d + 16u * gl;
                        if (x + 16 <= 1024) {
                            const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                            *reinterpret_cast<u32x4 *>(sp + x) = u32x4{lo.x, lo.y, hi.x, hi.y};
                        } else if (x + 8 == 1024) {
                            store8<NTS>(sp + x, piece(row, x));
                        }
                    }
                }
                return;
            }
    #pragma unroll SU
            for (int t = 0; t < 8; ++t) {
                const int cc = t * 8 + (lane >> 3);
                const uint64_t ci = c0 + (uint64_t)cc * CPL + j;
                if (!(wave_on && ci < a.N)) continue;
                const uint64_t rem = a.n - ci * 1024;
                const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
                const uint64_t base = soff[j & 1][wave][cc];
                uint8_t *sp = ob + base;
                const uint32_t *row = st + cc * RW;
                if (clen < 1024) {  // short last chunk of the object: this step's bytes, byte stores
                    const uint32_t *w = row + dofs(s) + 4 * gl;
                    for (int q = 0; q < 16; ++q) {
                        const uint32_t cb = 128u * s + 16u * gl + q;
                        if (cb < clen) sp[cb] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
                    }
                    continue;
                }
                // lines are aligned in memory, not in the stream: any 8-aligned object base
                const uint32_t d = (uint32_t)(-(uintptr_t)sp) & 127u;
                if (s >= 1) {  // the whole line [d + 128(s-1), d + 128 s)
                    const uint32_t x = d + 128u * (s - 1) + 16u * gl;
                    const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                    const u32x4 v = {lo.x, lo.y, hi.x, hi.y};
                    if (NTS) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(sp + x));
                    else *reinterpret_cast<u32x4 *>(sp + x) = v;
                } else {  // head [0, d): 8 B at 0 when d is 8 mod 16, then aligned 16-B pieces
                    const uint32_t h = d & 8u;
                    if (h && gl == 0) store8<NTS>(sp, piece(row, 0));
                    const uint32_t x = 16u * gl + h;
                    if (x + 16 <= d) {
                        const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                        *reinterpret_cast<u32x4 *>(sp + x) = u32x4{lo.x, lo.y, hi.x, hi.y};
                    }
                }
                if (s == 7) {  // tail [896 + d, 1024): aligned pieces, 8 B at the end
                    const uint32_t x = 896u + d + 16u * gl;
                    if (x + 16 <= 1024) {
                        const u32x2 lo = piece(row, x), hi = piece(row, x + 8);
                        const u32x4 v = {lo.x, lo.y, hi.x, hi.y};
                        *reinterpret_cast<u32x4 *>(sp + x) = v;
                    } else if (x + 8 == 1024) {
                        store8<NTS>(sp + x, piece(row, x));
                    }
                }
            }
        };

        uint32_t h[8];
    #pragma unroll
        for (int w = 0; w < 8; ++w) h[w] = IV(w);
        uint32_t L[LOG + 1][8];  // pending left nodes per level (CV stack)
        bool ok = true;
        // Verify-decode (CPL 2): the stored level-1 node of the lane's chunk
        // pair sits in the 64 bytes just before its first chunk, in lines the
        // step-0 loads fetch anyway.  Read it now, with them, instead of at
        // the pair's end (step 15), when those lines have long left L2 and
        // are fetched again (decode read 1.18x its stream).
        constexpr bool PN = MODE == 1 && CPL == 2 && BAO_DEC_PREFETCH && SE != 6;
        u32x4 pnode[4];
        if (PN && nmine == 2) {
            const uint8_t *np = ib + my_off - 64;
    #pragma unroll
            for (int q = 0; q < 4; ++q) pnode[q] = load16_a8(np + 16 * q);
        }

        u32x4 pre[8];
        load_step(0, pre);
        for (int g = 0; g < NSTEP; ++g) {
            const int j = g >> 3, s = g & 7;
    #pragma unroll
            for (int t = 0; t < 8; ++t) {
                uint32_t *row = st + (t * 8 + (lane >> 3)) * RW;
                if (MODE == 0 && SP == 0 && (lane & 7) == 7)  // carry the previous step's last 8 bytes
                    *reinterpret_cast<u32x2 *>(row + 2) = *reinterpret_cast<const u32x2 *>(row + ROW0 + 30);
                *reinterpret_cast<u32x4 *>(row + dofs(s) + (lane & 7) * 4) = pre[t];
            }
            if (MODE == 1 && ob) content_step(g, pre);
            if (MODE == 0 && ob && (SP == 1 || SP == 2)) stream_regs(g, pre);
            if (s == 7 && j + 1 < CPL) {  // stream offset of my next chunk, for the loads issued below
                const uint64_t ni = lb + j + 1;
                if ((uint64_t)(j + 1) < nmine) my_off += 1024 + 64 * (uint64_t)parents_at(ni, a.N);
                soff[(j + 1) & 1][wave][lane] = my_off;
            }
            wave_sync();
            if (MODE == 0 && ob && SP == 3 && SE == 1) stream_lines(g);
            if (g + 1 < NSTEP) load_step(g + 1, pre);  // in flight during the compressions
            if (MODE == 0 && ob && SP == 0) stream_step(wave, g);
            if (MODE == 0 && ob && SP == 3 && SE != 1) stream_lines(g);

            const uint64_t i = lb + j;
            const bool mine = (uint64_t)j < nmine;
            const uint32_t len = mine ? (uint32_t)((a.n - i * 1024) < 1024 ? (a.n - i * 1024) : 1024) : 0u;
            const uint32_t nb = len == 0 ? 1 : (len + 63) / 64;
            for (int hh = 0; hh < 2; ++hh) {
                const uint32_t b = (uint32_t)(2 * s + hh);
                if (mine && b < nb) {
                    uint32_t m[16];
                    const u32x4 *row = reinterpret_cast<const u32x4 *>(st + lane * RW + dofs(s) + hh * 16);
    #pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const u32x4 x = row[q];
                        m[4 * q] = x.x; m[4 * q + 1] = x.y; m[4 * q + 2] = x.z; m[4 * q + 3] = x.w;
                    }
                    const bool last = b + 1 == nb;
                    const uint32_t blen = last ? len - 64 * b : 64u;
                    const uint32_t flags = (b == 0 ? F_CHUNK_START : 0u) |
                                           (last ? (F_CHUNK_END | (a.N == 1 ? F_ROOT : 0u)) : 0u);
                    b3_compress(h, m, i, blen, flags);
                }
            }
            wave_sync();

            if (MODE == 2 && s == 7) {  // node check: chunk CV vs its stored slot (or the hash)
                if (mine) {
                    bool cok;
                    if (a.N == 1) {
                        const u32x4 *hp = reinterpret_cast<const u32x4 *>(a.hash + obj * 32);
                        const u32x4 e0 = hp[0], e1 = hp[1];
                        cok = e0.x == h[0] && e0.y == h[1] && e0.z == h[2] && e0.w == h[3] && e1.x == h[4] &&
                              e1.y == h[5] && e1.z == h[6] && e1.w == h[7];
                    } else {
                        cok = stored_slot_matches(ib, i, 0, a.N, h);
                    }
                    a.cv[obj * a.cv_stride + i] = cok ? 1 : 0;
                }
    #pragma unroll
                for (int w = 0; w < 8; ++w) h[w] = IV(w);
            } else if (s == 7) {  // chunk j of every lane is complete
                if (mine) {
                    const bool final = (uint64_t)j + 1 == nmine;
                    // CV stack: merge while the chunk count below this point is odd;
                    // on the lane's last chunk merge everything pending (promotions
                    // of a short tail follow the global tree)
                    bool done = false;
    #pragma unroll
                    for (int lv = 0; lv < LOG; ++lv) {
                        if (done) continue;
                        const bool bit = (j >> lv) & 1;
                        if (bit) {
                            const uint64_t sl = lb + ((uint64_t)(j >> (lv + 1)) << (lv + 1));
                            const bool root = a.N <= (2ull << lv);
                            if (PN && lv == 0) {  // the level-1 node read at step 0
                                const uint32_t *l = L[0];
                                ok &= pnode[0].x == l[0] && pnode[0].y == l[1] && pnode[0].z == l[2] &&
                                      pnode[0].w == l[3] && pnode[1].x == l[4] && pnode[1].y == l[5] &&
                                      pnode[1].z == l[6] && pnode[1].w == l[7] && pnode[2].x == h[0] &&
                                      pnode[2].y == h[1] && pnode[2].z == h[2] && pnode[2].w == h[3] &&
                                      pnode[3].x == h[4] && pnode[3].y == h[5] && pnode[3].z == h[6] &&
                                      pnode[3].w == h[7];
                            } else if (ob || MODE == 1) {
                                uint8_t *node = (MODE == 0 ? ob : const_cast<uint8_t *>(ib)) +
                                                parent_stream_off(sl, lv + 1, a.N);
                                ok &= node_io<MODE == 3 ? 0 : MODE, NTS>(node, L[lv], h);
                            }
                            uint32_t p[8];
                            b3_parent(L[lv], h, root, p);
    #pragma unroll
                            for (int w = 0; w < 8; ++w) h[w] = p[w];
                        } else if (!final) {
    #pragma unroll
                            for (int w = 0; w < 8; ++w) L[lv][w] = h[w];
                            done = true;
                        }
                    }
                    if (!done) {  // h is my level-LOG node (or the root)
                        if (a.N <= (uint64_t)CPL) {
                            root_io<MODE == 3 ? 0 : MODE>(a, obj, h);
                        } else {
                            u32x4 *cvp = reinterpret_cast<u32x4 *>(a.cv + (obj * a.cv_stride + lb / CPL) * 32);
                            cvp[0] = u32x4{h[0], h[1], h[2], h[3]};
                            cvp[1] = u32x4{h[4], h[5], h[6], h[7]};
                        }
                    }
                }
    #pragma unroll
                for (int w = 0; w < 8; ++w) h[w] = IV(w);
            }
        }
        if (MODE == 1 && !ok && SE != 6) flag_mismatch(a.status, obj);
        if (SE == 2 && diag == 0x9E3779B9u && ob) ob[0] = 0;  // keep the diagnostic's reads alive
        if (!DQ) break;
    }
    if (DQ && lane == 0) {  // the last wave out leaves the queue zero for the next launch
        const uint32_t done = atomicAdd(a.queue + 32, 1u);
        if (done + 1 == gridDim.x * (uint32_t)K3_WAVES) {
            a.queue[0] = 0u;
            a.queue[32] = 0u;
        }
    }
}

}  // namespace bao
}  // namespace chip

#include "bao_tree.hpp"  // the tree above the chunk CVs, and the K3 launchers
