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
#include <vector>

#include "../carbonado_amd/csrc/bao_device.hpp"

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

enum Op { ADD = 0, ADD3, XOR, BITOP3, ALIGNBIT, FMA, PERM, LSHLADD, NOPS };
static const char *op_name[NOPS] = {"v_add_u32", "v_add3_u32", "v_xor_b32", "v_bitop3_b32",
                                    "v_alignbit_b32", "v_fma_f32", "v_perm_b32", "v_lshl_add_u32"};

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
    probe_op<ADD>(iters);
    probe_op<ADD3>(iters);
    probe_op<XOR>(iters);
    probe_op<BITOP3>(iters);
    probe_op<ALIGNBIT>(iters);
    probe_op<FMA>(iters);
    probe_op<PERM>(iters);
    probe_op<LSHLADD>(iters);
    probe_b3<1>(iters / 64);
    probe_b3<2>(iters / 128);
    return 0;
}
