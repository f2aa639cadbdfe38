// layout_probe.hip — store-pattern calibration for writing zfec shards into
// bao chunk slots (K1-BL): 4 read + 8 write streams per object as K1, each
// wave writing one 1 KiB chunk per shard, with the chunk placed
//   0: shard-major (K1's layout, 128-B aligned chunks)
//   1: at its bao slot (8 mod 64), 16-B pieces shifted by 8 B (DPP) + 8-B head/tail stores
//   2: at its bao slot, but the wave writes the 8 whole memory lines starting at
//      the line holding the slot start + one 16-B piece (the planned line-owner scheme's
//      access pattern; data not meaningful)
// Calibration tool (not product code).   layout_probe [objects=1024]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../carbonado_amd/csrc/bao_device.hpp"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

struct Args {
    const uint8_t *in;
    uint8_t *out;
    const uint64_t *tab;
    uint64_t C, count, out_stride;
};

template <int MODE, int CH>
__global__ __launch_bounds__(256) void k_layout(Args a) {
    typedef const __attribute__((address_space(4))) uint64_t *ctab_t;
    const ctab_t tab = (ctab_t)a.tab;
    const uint64_t tpo = a.C / 4096, T = tpo * a.count;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    uint64_t c = (b % 8) * (G / 8) + b / 8, tin = 0;
    const int lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (;;) {
        if (tin == CH) { c += G; tin = 0; }
        const uint64_t t = c * CH + tin++;
        if (t >= T) break;
        const uint64_t obj = t / tpo;
        const uint64_t col = (t - obj * tpo) * 4096 + threadIdx.x * 16;
        const uint8_t *ib = a.in + obj * 4 * a.C;
        uint8_t *ob = a.out + obj * a.out_stride;
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *(const u32x4 *)(ib + j * a.C + col);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const u32x4 w = s < 4 ? v[s] : (v[s - 4] ^ 0x01020304u);
            const uint64_t p = (uint64_t)s * a.C + col;
            if (MODE == 0) {
                __builtin_nontemporal_store(w, (u32x4 *)(ob + p));
                continue;
            }
            const uint32_t ci = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 10));
            uint8_t *d = ob + tab[ci];
            if (MODE == 1) {
                const uint32_t nx = __builtin_amdgcn_update_dpp(0u, w.x, 0x130, 0xF, 0xF, false);
                const uint32_t ny = __builtin_amdgcn_update_dpp(0u, w.y, 0x130, 0xF, 0xF, false);
                if (lane < 63) __builtin_nontemporal_store(u32x4{w.z, w.w, nx, ny}, (u32x4 *)(d + 16 * lane + 8));
                if (lane == 0) __builtin_nontemporal_store(u32x2{w.x, w.y}, (u32x2 *)d);
                if (lane == 63) __builtin_nontemporal_store(u32x2{w.z, w.w}, (u32x2 *)(d + 1016));
            } else {
                uint8_t *l0 = (uint8_t *)((uintptr_t)d & ~(uintptr_t)127);
                __builtin_nontemporal_store(w, (u32x4 *)(l0 + 16 * lane));
                if (lane == 0) __builtin_nontemporal_store(w, (u32x4 *)(l0 + 1024));
            }
        }
    }
    (void)wv;
}

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 1024;
    const uint64_t n = 16ull << 20, C = n / 4, N = 2 * n / 1024;
    const uint64_t blen = 8 + 2 * n + 64 * (N - 1), bstride = (blen + 255) / 256 * 256;
    std::vector<uint64_t> h(N);
    for (uint64_t i = 0; i < N; ++i) h[i] = chip::bao::chunk_stream_off(i, N);
    uint8_t *in, *out;
    uint64_t *tab;
    CK(hipMalloc(&in, count * n));
    CK(hipMalloc(&out, count * bstride));
    CK(hipMalloc(&tab, N * 8));
    CK(hipMemcpy(tab, h.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemset(in, 7, count * n));
    CK(hipMemset(out, 0, count * bstride));
    struct V {
        const char *name;
        void (*fn)(Args);
        uint64_t stride;
    };
    std::vector<V> vs = {{"shard-major (K1)", k_layout<0, 64>, 2 * n},
                         {"bao slots, 8-B shifted pieces + head/tail", k_layout<1, 64>, bstride},
                         {"bao slots, whole memory lines", k_layout<2, 64>, bstride}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(vs.size());
    for (int rd = 0; rd < 5; ++rd)
        for (size_t i = 0; i < vs.size(); ++i) {
            Args a{in, out, tab, C, count, vs[i].stride};
            hipLaunchKernelGGL(vs[i].fn, dim3(1024), dim3(256), 0, 0, a);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(vs[i].fn, dim3(1024), dim3(256), 0, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto t = ms[i];
        std::sort(t.begin(), t.end());
        printf("%-46s median %7.3f ms -> %7.1f GB/s (48 MiB/object)\n", vs[i].name, t[2],
               3.0 * count * n / (t[2] * 1e-3) / 1e9);
    }
    return 0;
}
