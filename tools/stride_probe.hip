// stride_probe.hip — the product's 4-of-8 K1 kernel (schedule S0) on one pair
// of big allocations, with the object strides padded and the batch size
// varied, interleaved in ONE process so that the placement of the buffers in
// HBM is the same for every case (calibration tool, not product code).
//   stride_probe [rounds=5] [max_objects=2048]
// Cases: (objects, input pad, output pad) per line of the output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../carbonado_amd/csrc/gf256.hpp"
#include "zfec_variants.hpp"

using namespace chip;
using namespace chip::zf;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

namespace chip {
int num_cus() { return 256; }
}

__global__ void fill_kernel(uint64_t *p, size_t n, uint64_t seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        p[i] = z ^ (z >> 27);
    }
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const uint64_t maxobj = argc > 2 ? atoll(argv[2]) : 2048;
    const uint64_t n = 16ull << 20, C = n / 4;
    struct Case {
        uint64_t objects, pad_in, pad_out, base_obj;
    };
    const uint64_t KiB = 1024;
    std::vector<Case> cs = {{1024, 0, 0, 0},          {1024, 4 * KiB, 4 * KiB, 0}, {1024, 64 * KiB, 64 * KiB, 0},
                            {1024, 0, 0, 1024},       {2048, 0, 0, 0},           {1024, 1536 * KiB, 3 * 1024 * KiB, 0},
                            {512, 0, 0, 0}};
    uint64_t max_in = 0, max_out = 0;
    for (auto &c : cs) {
        max_in = std::max(max_in, (c.base_obj + c.objects) * (n + c.pad_in));
        max_out = std::max(max_out, (c.base_obj + c.objects) * (2 * n + c.pad_out));
    }
    if (maxobj < 2048) return 1;
    uint8_t *in, *out;
    CK(hipMalloc(&in, max_in));
    CK(hipMalloc(&out, max_out));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, max_in / 8, 0xCA4B0AD0ull);
    CK(hipMemset(out, 0, max_out));
    std::vector<uint8_t> enc = zfec_enc_matrix(4, 8);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(4 * 256, 0);
    for (int s = 0; s < 4; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < 4; ++r)
                tab[s * 256 + x] |= (uint32_t)gf.mul(enc[(4 + r) * 4 + s], (uint8_t)x) << (8 * r);
    uint32_t *dtab;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    auto fn = gf_apply_kernel<4, 1, 2, 3, true, 0, 2, 0, true>;  // the product's schedule S0
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(cs.size());
    for (int rd = 0; rd < rounds; ++rd)
        for (size_t i = 0; i < cs.size(); ++i) {
            const Case &c = cs[i];
            ApplyArgs a{};
            a.in = in + c.base_obj * (n + c.pad_in);
            a.out = out + c.base_obj * (2 * n + c.pad_out);
            a.in_stride = n + c.pad_in;
            a.out_stride = 2 * n + c.pad_out;
            a.valid = n;
            a.C = C;
            a.tiles_per_obj = C / TILE;
            a.total_tiles = a.tiles_per_obj * c.objects;
            a.count = c.objects;
            a.table = dtab;
            for (int j = 0; j < ZF_MAXK; ++j) {
                a.in_off[j] = j < 4 ? j * C : 0;
                a.copy_off[j] = j < 4 ? j * C : NO_OUT;
            }
            for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < 4 ? (4 + q) * C : NO_OUT;
            a.chunk = 32;  // ZF_CHUNK / U
            hipLaunchKernelGGL(fn, dim3(512), dim3(TPB), 256 * 4 * 8 * 4, 0, a);  // warm
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(fn, dim3(512), dim3(TPB), 256 * 4 * 8 * 4, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    for (size_t i = 0; i < cs.size(); ++i) {
        auto t = ms[i];
        std::sort(t.begin(), t.end());
        const double bytes = 3.0 * n * cs[i].objects;
        printf("objects %5llu pad_in %7llu KiB pad_out %7llu KiB base %5llu: median %7.3f ms -> %7.1f GB/s (%.4f of 8 TB/s)\n",
               (unsigned long long)cs[i].objects, (unsigned long long)(cs[i].pad_in / KiB),
               (unsigned long long)(cs[i].pad_out / KiB), (unsigned long long)cs[i].base_obj, t[t.size() / 2],
               bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / (t[t.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
