// valu_probe.hip — gfx950 int32 VALU issue rate, per instruction class and
// per waves/SIMD, and the BLAKE3 compression rate with one and with two
// independent states per lane.  Calibration tool: it settles the VALU peak
// that bench.py prices the bao / K13 / scrub rooflines against (VERDICT r2,
// "next round" item 1).
//
// Each lane runs 16 independent chains of one instruction (inline asm, so the
// compiler cannot fold or fuse them); a chained variant (one accumulator)
// gives the dependent latency.  Grid = 256 CUs x W blocks of 256 threads, i.e.
// W waves per SIMD when every block is resident (the kernels use few VGPRs).
// Every wave stamps s_memtime / s_memrealtime around its loop, so the report
// carries both the wall-clock rate (hipEvents) and cycles per instruction per
// wave (independent of the clock the chip holds).
//
//   valu_probe [iters=40000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../carbonado_amd/csrc/bao_device.hpp"
#include "b3g8_asm.h"

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

enum Op { ADD = 0, ADD3, XOR, BITOP3, ALIGNBIT, FMA, PERM, LSHLADD, XORSDWA, MIX, PKSWAP, LSHLOR, XAD, OR3, NOPS };
static const char *op_name[NOPS] = {"v_add_u32", "v_add3_u32", "v_xor_b32", "v_bitop3_b32",
                                    "v_alignbit_b32", "v_fma_f32", "v_perm_b32", "v_lshl_add_u32",
                                    "v_xor_b32_sdwa", "mix4", "v_pk_add_u16 swap", "v_lshl_or_b32",
                                    "v_xad_u32", "v_or3_b32"};

template <int OP>
__device__ __forceinline__ void one(uint32_t &x, uint32_t a, uint32_t b) {
    if constexpr (OP == ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == ADD3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
    if constexpr (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == LSHLADD) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == XORSDWA)
        asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
                     : "+v"(x) : "v"(a));
    // round 4: rotate-by-16 as a packed 16-bit add with swapped halves (x.hi + 0 | x.lo + 0 << 16),
    // and three more VOP3 integer forms
    if constexpr (OP == PKSWAP) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,0]" : "+v"(x));
    if constexpr (OP == LSHLOR) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(a));
    if constexpr (OP == XAD) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    if constexpr (OP == OR3) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    // one of each class on the chain in BLAKE3's G order: counted as 4 instructions
    if constexpr (OP == MIX) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(a));
        asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
    }
}

struct Stamp { uint64_t t0, t1, r0, r1; };

// CH independent chains, 64 instructions per loop iteration.
template <int OP, int CH>
__global__ __launch_bounds__(256) void chain_kernel(uint32_t *out, Stamp *st, int iters, uint32_t a, uint32_t b) {
    uint32_t x[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * 7u + i;
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 64 / CH; ++u)
#pragma unroll
            for (int i = 0; i < CH; ++i) one<OP>(x[i], a, b);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        Stamp v{t0, t1, r0, r1};
        st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = v;
    }
}

// The mix4 instructions grouped by class: 16 chains, each class applied to
// all 16 before the next class (64 instructions per loop iteration, the same
// multiset as mix4's).
__global__ __launch_bounds__(256) void mixg_kernel(uint32_t *out, Stamp *st, int iters, uint32_t a, uint32_t b) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 7u + i;
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x[i]));
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        Stamp v{t0, t1, r0, r1};
        st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = v;
    }
}

// NS independent BLAKE3 compressions per lane per iteration (the product's
// b3_compress: 7 rounds x 8 G, 12 VALU per G = 672 per compression).
template <int NS>
__global__ __launch_bounds__(256) void b3_kernel(uint32_t *out, Stamp *st, int iters, uint32_t seed) {
    uint32_t h[NS][8], m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = seed * (i + 1) + threadIdx.x;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i) h[s][i] = chip::bao::IV(i) + s + threadIdx.x;
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < NS; ++s) chip::bao::b3_compress(h[s], m, (uint64_t)it, 64, 0);
        m[it & 15] ^= h[0][it & 7];  // keep the message live (one op per iteration)
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) s ^= h[q][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        Stamp v{t0, t1, r0, r1};
        st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = v;
    }
}

__device__ __forceinline__ uint32_t xor_rot16(uint32_t d, uint32_t a) {
    uint32_t r;
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1"
                 : "=v"(r) : "v"(d), "v"(a));
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
                 : "+v"(r) : "v"(d), "v"(a));
    return r;
}
__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b, uint32_t m) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2\n\tv_add_u32 %0, %0, %3" : "=&v"(r) : "v"(a), "v"(b), "v"(m));
    return r;
}
template <int VAR>
__device__ __forceinline__ void gv(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t x, uint32_t y) {
    a = VAR == 2 ? add2(a, b, x) : a + b + x;
    d = VAR >= 1 ? xor_rot16(d, a) : chip::bao::rotr(d ^ a, 16);
    c = c + d;
    b = chip::bao::rotr(b ^ c, 12);
    a = VAR == 2 ? add2(a, b, y) : a + b + y;
    d = chip::bao::rotr(d ^ a, 8);
    c = c + d;
    b = chip::bao::rotr(b ^ c, 7);
}
#define ADD3(d, x, y) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(d) : "v"(x), "v"(y))
#define XOR(d, x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(d) : "v"(x))
#define ROT(d, n) asm volatile("v_alignbit_b32 %0, %0, %0, " #n : "+v"(d))
#define ADD(d, x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(x))
// four G's at once, each step applied to the four before the next step
__device__ __forceinline__ void g4(uint32_t &a0, uint32_t &b0, uint32_t &c0, uint32_t &d0, uint32_t &a1, uint32_t &b1,
                                   uint32_t &c1, uint32_t &d1, uint32_t &a2, uint32_t &b2, uint32_t &c2, uint32_t &d2,
                                   uint32_t &a3, uint32_t &b3, uint32_t &c3, uint32_t &d3, uint32_t x0, uint32_t y0,
                                   uint32_t x1, uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) {
    ADD3(a0, b0, x0); ADD3(a1, b1, x1); ADD3(a2, b2, x2); ADD3(a3, b3, x3);
    XOR(d0, a0); XOR(d1, a1); XOR(d2, a2); XOR(d3, a3);
    ROT(d0, 16); ROT(d1, 16); ROT(d2, 16); ROT(d3, 16);
    ADD(c0, d0); ADD(c1, d1); ADD(c2, d2); ADD(c3, d3);
    XOR(b0, c0); XOR(b1, c1); XOR(b2, c2); XOR(b3, c3);
    ROT(b0, 12); ROT(b1, 12); ROT(b2, 12); ROT(b3, 12);
    ADD3(a0, b0, y0); ADD3(a1, b1, y1); ADD3(a2, b2, y2); ADD3(a3, b3, y3);
    XOR(d0, a0); XOR(d1, a1); XOR(d2, a2); XOR(d3, a3);
    ROT(d0, 8); ROT(d1, 8); ROT(d2, 8); ROT(d3, 8);
    ADD(c0, d0); ADD(c1, d1); ADD(c2, d2); ADD(c3, d3);
    XOR(b0, c0); XOR(b1, c1); XOR(b2, c2); XOR(b3, c3);
    ROT(b0, 7); ROT(b1, 7); ROT(b2, 7); ROT(b3, 7);
}
// One asm statement per four G's with SEP between the 12 groups of four
// (VAR 4: "s_nop 0", VAR 5: "s_nop 1", VAR 6: nothing, VAR 7: s_nop 0 after
// the VOP2 groups only, VAR 8: after the VOP3 groups only): does the hazard recognizer's s_nop between dependent
// groups (VAR 3) cost or help?
#define G4B(S3, S2)                                                                                   \
    "v_add3_u32 %0, %0, %4, %16\n\tv_add3_u32 %1, %1, %5, %17\n\tv_add3_u32 %2, %2, %6, %18\n\t"    \
    "v_add3_u32 %3, %3, %7, %19\n\t" S3                                                               \
    "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\t" S2 \
    "v_alignbit_b32 %12, %12, %12, 16\n\tv_alignbit_b32 %13, %13, %13, 16\n\t"                          \
    "v_alignbit_b32 %14, %14, %14, 16\n\tv_alignbit_b32 %15, %15, %15, 16\n\t" S3                        \
    "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\t" S2 \
    "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\t" S2 \
    "v_alignbit_b32 %4, %4, %4, 12\n\tv_alignbit_b32 %5, %5, %5, 12\n\t"                                \
    "v_alignbit_b32 %6, %6, %6, 12\n\tv_alignbit_b32 %7, %7, %7, 12\n\t" S3                              \
    "v_add3_u32 %0, %0, %4, %20\n\tv_add3_u32 %1, %1, %5, %21\n\tv_add3_u32 %2, %2, %6, %22\n\t"    \
    "v_add3_u32 %3, %3, %7, %23\n\t" S3                                                               \
    "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\t" S2 \
    "v_alignbit_b32 %12, %12, %12, 8\n\tv_alignbit_b32 %13, %13, %13, 8\n\t"                            \
    "v_alignbit_b32 %14, %14, %14, 8\n\tv_alignbit_b32 %15, %15, %15, 8\n\t" S3                          \
    "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\t" S2 \
    "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\t" S2 \
    "v_alignbit_b32 %4, %4, %4, 7\n\tv_alignbit_b32 %5, %5, %5, 7\n\t"                                  \
    "v_alignbit_b32 %6, %6, %6, 7\n\tv_alignbit_b32 %7, %7, %7, 7"
#define G4A(SEP) G4B(SEP, SEP)
// VAR 13 / 14 (round 4): the rotate by 16 as v_pk_add_u16 with swapped halves
// (S16 after it: VAR 13 none, VAR 14 "s_nop 0"); nops after the VOP2 groups as VAR 7
#define G4P(S16)                                                                                      \
    "v_add3_u32 %0, %0, %4, %16\n\tv_add3_u32 %1, %1, %5, %17\n\tv_add3_u32 %2, %2, %6, %18\n\t"    \
    "v_add3_u32 %3, %3, %7, %19\n\t"                                                                  \
    "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\ts_nop 0\n\t" \
    "v_pk_add_u16 %12, %12, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\tv_pk_add_u16 %13, %13, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\t" \
    "v_pk_add_u16 %14, %14, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\tv_pk_add_u16 %15, %15, 0 op_sel:[1,0] op_sel_hi:[0,0]\n\t" S16 \
    "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\ts_nop 0\n\t" \
    "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\ts_nop 0\n\t" \
    "v_alignbit_b32 %4, %4, %4, 12\n\tv_alignbit_b32 %5, %5, %5, 12\n\t"                                \
    "v_alignbit_b32 %6, %6, %6, 12\n\tv_alignbit_b32 %7, %7, %7, 12\n\t"                                \
    "v_add3_u32 %0, %0, %4, %20\n\tv_add3_u32 %1, %1, %5, %21\n\tv_add3_u32 %2, %2, %6, %22\n\t"    \
    "v_add3_u32 %3, %3, %7, %23\n\t"                                                                  \
    "v_xor_b32 %12, %12, %0\n\tv_xor_b32 %13, %13, %1\n\tv_xor_b32 %14, %14, %2\n\tv_xor_b32 %15, %15, %3\n\ts_nop 0\n\t" \
    "v_alignbit_b32 %12, %12, %12, 8\n\tv_alignbit_b32 %13, %13, %13, 8\n\t"                            \
    "v_alignbit_b32 %14, %14, %14, 8\n\tv_alignbit_b32 %15, %15, %15, 8\n\t"                            \
    "v_add_u32 %8, %8, %12\n\tv_add_u32 %9, %9, %13\n\tv_add_u32 %10, %10, %14\n\tv_add_u32 %11, %11, %15\n\ts_nop 0\n\t" \
    "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %9\n\tv_xor_b32 %6, %6, %10\n\tv_xor_b32 %7, %7, %11\n\ts_nop 0\n\t" \
    "v_alignbit_b32 %4, %4, %4, 7\n\tv_alignbit_b32 %5, %5, %5, 7\n\t"                                  \
    "v_alignbit_b32 %6, %6, %6, 7\n\tv_alignbit_b32 %7, %7, %7, 7"
template <int NOPK>
__device__ __forceinline__ void g4a(uint32_t &a0, uint32_t &b0, uint32_t &c0, uint32_t &d0, uint32_t &a1, uint32_t &b1,
                                    uint32_t &c1, uint32_t &d1, uint32_t &a2, uint32_t &b2, uint32_t &c2, uint32_t &d2,
                                    uint32_t &a3, uint32_t &b3, uint32_t &c3, uint32_t &d3, uint32_t x0, uint32_t y0,
                                    uint32_t x1, uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) {
#define G4A_OPS                                                                                        \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(c0), "+v"(c1), \
      "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)                                      \
    : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(y0), "v"(y1), "v"(y2), "v"(y3)
    if constexpr (NOPK == 13) asm volatile(G4P("") G4A_OPS);
    else if constexpr (NOPK == 14) asm volatile(G4P("s_nop 0\n\t") G4A_OPS);
    else if constexpr (NOPK == 0) asm volatile(G4A("s_nop 0\n\t") G4A_OPS);
    else if constexpr (NOPK == 1) asm volatile(G4A("s_nop 1\n\t") G4A_OPS);
    else if constexpr (NOPK == 2) asm volatile(G4B("", "s_nop 0\n\t") G4A_OPS);  // after VOP2 groups only
    else if constexpr (NOPK == 3) asm volatile(G4B("s_nop 0\n\t", "") G4A_OPS);  // after VOP3 groups only
    else asm volatile(G4A("") G4A_OPS);
#undef G4A_OPS
}
template <int VAR, int R>
__device__ __forceinline__ void rv(uint32_t (&v)[16], const uint32_t (&m)[16]) {
    using chip::bao::SCHED;
    if constexpr (VAR >= 4) {
        constexpr int K = VAR == 4 ? 0 : VAR == 5 ? 1 : VAR == 7 ? 2 : VAR == 8 ? 3 : VAR >= 13 ? VAR : -1;
        g4a<K>(v[0], v[4], v[8], v[12], v[1], v[5], v[9], v[13], v[2], v[6], v[10], v[14], v[3], v[7], v[11], v[15],
               m[SCHED(R, 0)], m[SCHED(R, 1)], m[SCHED(R, 2)], m[SCHED(R, 3)], m[SCHED(R, 4)], m[SCHED(R, 5)],
               m[SCHED(R, 6)], m[SCHED(R, 7)]);
        g4a<K>(v[0], v[5], v[10], v[15], v[1], v[6], v[11], v[12], v[2], v[7], v[8], v[13], v[3], v[4], v[9], v[14],
               m[SCHED(R, 8)], m[SCHED(R, 9)], m[SCHED(R, 10)], m[SCHED(R, 11)], m[SCHED(R, 12)], m[SCHED(R, 13)],
               m[SCHED(R, 14)], m[SCHED(R, 15)]);
        return;
    }
    if constexpr (VAR == 3) {
        g4(v[0], v[4], v[8], v[12], v[1], v[5], v[9], v[13], v[2], v[6], v[10], v[14], v[3], v[7], v[11], v[15],
           m[SCHED(R, 0)], m[SCHED(R, 1)], m[SCHED(R, 2)], m[SCHED(R, 3)], m[SCHED(R, 4)], m[SCHED(R, 5)],
           m[SCHED(R, 6)], m[SCHED(R, 7)]);
        g4(v[0], v[5], v[10], v[15], v[1], v[6], v[11], v[12], v[2], v[7], v[8], v[13], v[3], v[4], v[9], v[14],
           m[SCHED(R, 8)], m[SCHED(R, 9)], m[SCHED(R, 10)], m[SCHED(R, 11)], m[SCHED(R, 12)], m[SCHED(R, 13)],
           m[SCHED(R, 14)], m[SCHED(R, 15)]);
        return;
    }
    gv<VAR>(v[0], v[4], v[8], v[12], m[SCHED(R, 0)], m[SCHED(R, 1)]);
    gv<VAR>(v[1], v[5], v[9], v[13], m[SCHED(R, 2)], m[SCHED(R, 3)]);
    gv<VAR>(v[2], v[6], v[10], v[14], m[SCHED(R, 4)], m[SCHED(R, 5)]);
    gv<VAR>(v[3], v[7], v[11], v[15], m[SCHED(R, 6)], m[SCHED(R, 7)]);
    gv<VAR>(v[0], v[5], v[10], v[15], m[SCHED(R, 8)], m[SCHED(R, 9)]);
    gv<VAR>(v[1], v[6], v[11], v[12], m[SCHED(R, 10)], m[SCHED(R, 11)]);
    gv<VAR>(v[2], v[7], v[8], v[13], m[SCHED(R, 12)], m[SCHED(R, 13)]);
    gv<VAR>(v[3], v[4], v[9], v[14], m[SCHED(R, 14)], m[SCHED(R, 15)]);
}
template <int VAR>
__device__ __forceinline__ void cv_compress(uint32_t (&h)[8], const uint32_t (&m)[16], uint64_t ctr, uint32_t blen,
                                            uint32_t flags) {
    using chip::bao::IV;
    uint32_t v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], IV(0), IV(1), IV(2), IV(3),
                      (uint32_t)ctr, (uint32_t)(ctr >> 32), blen, flags};
    rv<VAR, 0>(v, m); rv<VAR, 1>(v, m); rv<VAR, 2>(v, m); rv<VAR, 3>(v, m);
    rv<VAR, 4>(v, m); rv<VAR, 5>(v, m); rv<VAR, 6>(v, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = v[i] ^ v[i + 8];
}
// BLAKE3 variants: VAR 1 = rot16 fused into its xor as two SDWA xors, VAR 2 =
// VAR 1 + a+b+m as two v_add_u32 instead of v_add3_u32.  out[] of every
// variant must equal VAR 0's (checked on the host).
template <int VAR>
__global__ __launch_bounds__(256) void b3v_kernel(uint32_t *out, Stamp *st, int iters, uint32_t seed) {
    uint32_t h[8], m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = seed * (i + 1) + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = chip::bao::IV(i) + threadIdx.x;
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        cv_compress<VAR>(h, m, (uint64_t)it, 64, 0);
        m[it & 15] ^= h[it & 7];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= h[i] * (i + 1);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        Stamp v{t0, t1, r0, r1};
        st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = v;
    }
}

struct Result { double ms, lane_ops_t, cyc_per_inst_wave, clock_ghz; };

template <typename L>
static Result run(L launch, int W, double insts_per_lane, int reps) {
    const int blocks = 256 * W, threads = blocks * 256, waves = threads / 64;
    static uint32_t *d_out = nullptr;
    static Stamp *d_st = nullptr;
    if (!d_out) {
        CK(hipMalloc(&d_out, 256 * 8 * 256 * 4));
        CK(hipMalloc(&d_st, 256 * 8 * 4 * sizeof(Stamp)));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch(blocks, d_out, d_st);  // warm-up
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    std::vector<Stamp> st(waves);
    double cyc = 0, clk = 0;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        launch(blocks, d_out, d_st);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) {
            best = ms;
            CK(hipMemcpy(st.data(), d_st, waves * sizeof(Stamp), hipMemcpyDeviceToHost));
            std::vector<double> c(waves), g(waves);
            for (int w = 0; w < waves; ++w) {
                c[w] = (double)(st[w].t1 - st[w].t0);
                g[w] = c[w] / ((double)(st[w].r1 - st[w].r0) * 10.0);  // realtime = 100 MHz -> GHz
            }
            std::sort(c.begin(), c.end());
            std::sort(g.begin(), g.end());
            cyc = c[waves / 2];
            clk = g[waves / 2];
        }
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    Result res;
    res.ms = best;
    res.lane_ops_t = (double)threads * insts_per_lane / (best * 1e-3) / 1e12;
    res.cyc_per_inst_wave = cyc / insts_per_lane;
    res.clock_ghz = clk;
    return res;
}

template <int OP>
static void probe_op(int iters) {
    for (int W : {1, 2, 4, 8}) {
        Result r = run([&](int blocks, uint32_t *o, Stamp *s) {
            chain_kernel<OP, 16><<<blocks, 256>>>(o, s, iters, 0x9E3779B9u, 0x85EBCA6Bu);
        }, W, 64.0 * iters, 3);
        printf("%-16s indep16 W=%d  %8.3f ms  %7.2f T lane-op/s  %6.2f cyc/inst/wave  %5.2f cyc/inst/SIMD  clk %.2f GHz\n",
               op_name[OP], W, r.ms, r.lane_ops_t, r.cyc_per_inst_wave, r.cyc_per_inst_wave / W, r.clock_ghz);
    }
    Result r = run([&](int blocks, uint32_t *o, Stamp *s) {
        chain_kernel<OP, 1><<<blocks, 256>>>(o, s, iters / 4, 0x9E3779B9u, 0x85EBCA6Bu);
    }, 1, 64.0 * (iters / 4), 3);
    printf("%-16s chain1  W=1  %8.3f ms  %7.2f T lane-op/s  %6.2f cyc/inst/wave (dependent latency)\n",
           op_name[OP], r.ms, r.lane_ops_t, r.cyc_per_inst_wave);
    fflush(stdout);
}

// Two independent compressions per lane, their eight G's advanced step by
// step as one asm statement per half-round (VAR 10: no nops, 11: s_nop 0
// after the VOP2 groups), against the compiler's own interleaving of two
// plain-C compressions (VAR 12).  Counted as 2 compressions per iteration.
template <int VAR>
__device__ __forceinline__ void g8(uint32_t (&v)[16], uint32_t (&u)[16], const uint32_t *m, const uint32_t *n, int i0,
                                   int i1, int i2, int i3, int j0, int j1, int j2, int j3, int k0, int k1, int k2,
                                   int k3, int l0, int l1, int l2, int l3, int x0, int y0, int x1, int y1, int x2, int y2,
                                   int x3, int y3) {
#define G8_OPS                                                                                                 \
    : "+v"(v[i0]), "+v"(v[i1]), "+v"(v[i2]), "+v"(v[i3]), "+v"(v[j0]), "+v"(v[j1]), "+v"(v[j2]), "+v"(v[j3]),   \
      "+v"(v[k0]), "+v"(v[k1]), "+v"(v[k2]), "+v"(v[k3]), "+v"(v[l0]), "+v"(v[l1]), "+v"(v[l2]), "+v"(v[l3]),   \
      "+v"(u[i0]), "+v"(u[i1]), "+v"(u[i2]), "+v"(u[i3]), "+v"(u[j0]), "+v"(u[j1]), "+v"(u[j2]), "+v"(u[j3]),   \
      "+v"(u[k0]), "+v"(u[k1]), "+v"(u[k2]), "+v"(u[k3]), "+v"(u[l0]), "+v"(u[l1]), "+v"(u[l2]), "+v"(u[l3])    \
    : "v"(m[x0]), "v"(m[x1]), "v"(m[x2]), "v"(m[x3]), "v"(n[x0]), "v"(n[x1]), "v"(n[x2]), "v"(n[x3]),           \
      "v"(m[y0]), "v"(m[y1]), "v"(m[y2]), "v"(m[y3]), "v"(n[y0]), "v"(n[y1]), "v"(n[y2]), "v"(n[y3])
    if constexpr (VAR == 10) asm volatile(G8ASM_PLAIN G8_OPS);
    else asm volatile(G8ASM_NOP G8_OPS);
#undef G8_OPS
}
template <int VAR, int R>
__device__ __forceinline__ void r2(uint32_t (&v)[16], uint32_t (&u)[16], const uint32_t (&m)[16], const uint32_t (&n)[16]) {
    using chip::bao::SCHED;
    using chip::bao::rotr;
    if constexpr (VAR == 12) {
        B3G(v[0], v[4], v[8], v[12], m[SCHED(R, 0)], m[SCHED(R, 1)]);
        B3G(u[0], u[4], u[8], u[12], n[SCHED(R, 0)], n[SCHED(R, 1)]);
        B3G(v[1], v[5], v[9], v[13], m[SCHED(R, 2)], m[SCHED(R, 3)]);
        B3G(u[1], u[5], u[9], u[13], n[SCHED(R, 2)], n[SCHED(R, 3)]);
        B3G(v[2], v[6], v[10], v[14], m[SCHED(R, 4)], m[SCHED(R, 5)]);
        B3G(u[2], u[6], u[10], u[14], n[SCHED(R, 4)], n[SCHED(R, 5)]);
        B3G(v[3], v[7], v[11], v[15], m[SCHED(R, 6)], m[SCHED(R, 7)]);
        B3G(u[3], u[7], u[11], u[15], n[SCHED(R, 6)], n[SCHED(R, 7)]);
        B3G(v[0], v[5], v[10], v[15], m[SCHED(R, 8)], m[SCHED(R, 9)]);
        B3G(u[0], u[5], u[10], u[15], n[SCHED(R, 8)], n[SCHED(R, 9)]);
        B3G(v[1], v[6], v[11], v[12], m[SCHED(R, 10)], m[SCHED(R, 11)]);
        B3G(u[1], u[6], u[11], u[12], n[SCHED(R, 10)], n[SCHED(R, 11)]);
        B3G(v[2], v[7], v[8], v[13], m[SCHED(R, 12)], m[SCHED(R, 13)]);
        B3G(u[2], u[7], u[8], u[13], n[SCHED(R, 12)], n[SCHED(R, 13)]);
        B3G(v[3], v[4], v[9], v[14], m[SCHED(R, 14)], m[SCHED(R, 15)]);
        B3G(u[3], u[4], u[9], u[14], n[SCHED(R, 14)], n[SCHED(R, 15)]);
        return;
    }
    g8<VAR>(v, u, m, n, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, SCHED(R, 0), SCHED(R, 1), SCHED(R, 2),
            SCHED(R, 3), SCHED(R, 4), SCHED(R, 5), SCHED(R, 6), SCHED(R, 7));
    g8<VAR>(v, u, m, n, 0, 1, 2, 3, 5, 6, 7, 4, 10, 11, 8, 9, 15, 12, 13, 14, SCHED(R, 8), SCHED(R, 9), SCHED(R, 10),
            SCHED(R, 11), SCHED(R, 12), SCHED(R, 13), SCHED(R, 14), SCHED(R, 15));
}
template <int VAR>
__global__ __launch_bounds__(256) void b3x2_kernel(uint32_t *out, Stamp *st, int iters, uint32_t seed) {
    using chip::bao::IV;
    uint32_t h[8], g[8], m[16], n[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { m[i] = seed * (i + 1) + threadIdx.x; n[i] = m[i] ^ 0x5A5A5A5Au; }
#pragma unroll
    for (int i = 0; i < 8; ++i) { h[i] = IV(i) + threadIdx.x; g[i] = IV(i) + 7 * threadIdx.x; }
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        uint32_t v[16] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], IV(0), IV(1), IV(2), IV(3),
                          (uint32_t)it, 0u, 64u, 0u};
        uint32_t u[16] = {g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], IV(0), IV(1), IV(2), IV(3),
                          (uint32_t)it, 1u, 64u, 0u};
        r2<VAR, 0>(v, u, m, n); r2<VAR, 1>(v, u, m, n); r2<VAR, 2>(v, u, m, n); r2<VAR, 3>(v, u, m, n);
        r2<VAR, 4>(v, u, m, n); r2<VAR, 5>(v, u, m, n); r2<VAR, 6>(v, u, m, n);
#pragma unroll
        for (int i = 0; i < 8; ++i) { h[i] = v[i] ^ v[i + 8]; g[i] = u[i] ^ u[i + 8]; }
        m[it & 15] ^= h[it & 7];
        n[it & 15] ^= g[it & 7];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= h[i] ^ g[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        Stamp q{t0, t1, r0, r1};
        st[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = q;
    }
}
template <int VAR>
static void probe_b3x2(int iters, std::vector<uint32_t> *ref) {
    for (int W : {1, 2, 3, 4, 8}) {
        Result r = run([&](int blocks, uint32_t *o, Stamp *s) { b3x2_kernel<VAR><<<blocks, 256>>>(o, s, iters, 12345u); },
                       W, 2 * 672.0 * iters, 3);
        printf("blake3 x2 interleaved VAR %d W=%d  %8.3f ms  %7.2f T lane-op/s (672/compress)  %.3e compress/s  clk %.2f GHz\n",
               VAR, W, r.ms, r.lane_ops_t, r.lane_ops_t * 1e12 / 672.0, r.clock_ghz);
    }
    uint32_t *d = nullptr;
    Stamp *st = nullptr;
    CK(hipMalloc(&d, 256 * 256 * 4));
    CK(hipMalloc(&st, 256 * 4 * sizeof(Stamp)));
    b3x2_kernel<VAR><<<256, 256>>>(d, st, 50, 777u);
    std::vector<uint32_t> h(256 * 256);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    if (ref->empty()) *ref = h;
    printf("blake3 x2 VAR %d output %s VAR 12\n", VAR, h == *ref ? "==" : "!=");
    CK(hipFree(d));
    CK(hipFree(st));
    fflush(stdout);
}

template <int VAR>
static void probe_b3v(int iters, std::vector<uint32_t> *ref) {
    for (int W : {2, 3, 4, 8}) {
        Result r = run([&](int blocks, uint32_t *o, Stamp *s) {
            b3v_kernel<VAR><<<blocks, 256>>>(o, s, iters, 12345u);
        }, W, 672.0 * iters, 3);
        printf("blake3 VAR %d W=%d  %8.3f ms  %7.2f T lane-op/s (672/compress)  %.3e compress/s  clk %.2f GHz\n", VAR,
               W, r.ms, r.lane_ops_t, r.lane_ops_t * 1e12 / 672.0, r.clock_ghz);
    }
    // correctness of the variant: one W=1 launch's outputs against VAR 0's
    uint32_t *d = nullptr;
    Stamp *st = nullptr;
    CK(hipMalloc(&d, 256 * 256 * 4));
    CK(hipMalloc(&st, 256 * 4 * sizeof(Stamp)));
    b3v_kernel<VAR><<<256, 256>>>(d, st, 50, 777u);
    std::vector<uint32_t> h(256 * 256);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    if (ref->empty()) *ref = h;
    printf("blake3 VAR %d output %s VAR 0\n", VAR, h == *ref ? "==" : "!=");
    CK(hipFree(d));
    CK(hipFree(st));
    fflush(stdout);
}

template <int NS>
static void probe_b3(int iters) {
    for (int W : {1, 2, 3, 4, 8}) {
        Result r = run([&](int blocks, uint32_t *o, Stamp *s) {
            b3_kernel<NS><<<blocks, 256>>>(o, s, iters, 12345u);
        }, W, 672.0 * NS * iters, 3);
        printf("blake3 x%d states W=%d  %8.3f ms  %7.2f T lane-op/s (672/compress)  %6.1f cyc/compress/wave  "
               "%6.1f cyc/compress/SIMD  %.3e compress/s  clk %.2f GHz\n",
               NS, W, r.ms, r.lane_ops_t, r.cyc_per_inst_wave * 672.0, r.cyc_per_inst_wave * 672.0 / W,
               r.lane_ops_t * 1e12 / 672.0, r.clock_ghz);
    }
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 40000;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("device %s, %d CUs, clockRate %d kHz; nominal: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.64 T lane-op/s "
           "(2-cycle wave64 issue), 39.32 at 4 cycles\n",
           p.gcnArchName, p.multiProcessorCount, p.clockRate);
    // argv[2] == "b3": only the BLAKE3 rows (x1/x2 states = the product's b3_compress)
    const bool b3only = argc > 2 && std::string(argv[2]) == "b3";
    if (!b3only) {
    probe_op<ADD>(iters);
    probe_op<ADD3>(iters);
    probe_op<XOR>(iters);
    probe_op<BITOP3>(iters);
    probe_op<ALIGNBIT>(iters);
    probe_op<FMA>(iters);
    probe_op<PERM>(iters);
    probe_op<LSHLADD>(iters);
    probe_op<XORSDWA>(iters);
    probe_op<MIX>(iters / 4);
    for (int W : {2, 4, 8}) {
        Result r = run([&](int blocks, uint32_t *o, Stamp *s) {
            mixg_kernel<<<blocks, 256>>>(o, s, iters / 4, 0x9E3779B9u, 0x85EBCA6Bu);
        }, W, 64.0 * (iters / 4), 3);
        printf("mix4 grouped     W=%d  %8.3f ms  %7.2f T lane-instr/s  (mix4 row: ops counted in groups of 4)\n", W,
               r.ms, r.lane_ops_t);
    }
    }
    std::vector<uint32_t> ref;
    if (argc > 2 && std::string(argv[2]) == "pk") {  // round 4: rot16 as a packed swap (VAR 13/14 vs 7)
        probe_op<PKSWAP>(iters);
        probe_op<ALIGNBIT>(iters);
        probe_op<LSHLOR>(iters);
        probe_op<XAD>(iters);
        probe_op<OR3>(iters);
        probe_b3v<0>(iters / 64, &ref);
        probe_b3v<7>(iters / 64, &ref);
        probe_b3v<13>(iters / 64, &ref);
        probe_b3v<14>(iters / 64, &ref);
        probe_b3v<7>(iters / 64, &ref);
        probe_b3v<13>(iters / 64, &ref);
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "b3x2") {  // two states per lane (VAR 10-12)
        probe_b3v<0>(iters / 64, &ref);
        probe_b3v<7>(iters / 64, &ref);
        std::vector<uint32_t> ref2;
        probe_b3x2<12>(iters / 128, &ref2);
        probe_b3x2<10>(iters / 128, &ref2);
        probe_b3x2<11>(iters / 128, &ref2);
        probe_b3v<7>(iters / 64, &ref);
        return 0;
    }
    if (b3only) {  // warm the clock up, then the variants back to back
        probe_b3v<0>(iters / 64, &ref);
        probe_b3v<3>(iters / 64, &ref);
        probe_b3v<4>(iters / 64, &ref);
        probe_b3v<5>(iters / 64, &ref);
        probe_b3v<6>(iters / 64, &ref);
        probe_b3v<7>(iters / 64, &ref);
        probe_b3v<8>(iters / 64, &ref);
        probe_b3v<3>(iters / 64, &ref);
        probe_b3<1>(iters / 64);
        return 0;
    }
    probe_b3<1>(iters / 64);
    probe_b3<2>(iters / 128);
    probe_b3v<0>(iters / 64, &ref);
    probe_b3v<1>(iters / 64, &ref);
    probe_b3v<2>(iters / 64, &ref);
    probe_b3v<3>(iters / 64, &ref);
    return 0;
}
