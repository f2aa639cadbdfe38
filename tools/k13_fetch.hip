// k13_fetch.hip — read-traffic attribution of K13's general path (VERDICT r4
// item 2: raw FETCH_SIZE per launch +21 % over the FULL path for the same
// input bytes).  Runs, in one process and in a fixed order, the FULL product
// kernel at the 16 MiB shape (4096 chunk-columns per shard) and the general
// product kernel at the 16 MiB shape and at the level-15 shape (4097
// columns, zfec padding), plus diagnostics (fused_device.hpp DG 1, 3, 5, 11,
// 12, 13, 14), each `reps` times after one warm-up launch.  Under
// `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` the dispatches come out
// in this order; tools/k13_fetch_summary.py pairs them with the labels this
// prints.  Calibration tool (not product code).
//   k13_fetch [objects=256] [reps=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fused_variants.hpp"
#include "../carbonado_amd/csrc/gf256.hpp"
#include "../carbonado_amd/csrc/hbm_alloc.hpp"

using namespace chip;

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
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct Shape {
    const char *name;
    uint64_t n, C, cols, N, bpo, in_stride, out_stride;
    uint64_t *coff;
};

// in_align: the input rows' stride alignment (256, or 16: the C-ABI's minimum,
// which bench.py's pipeline rows used for n = 16779371)
static Shape make_shape(const char *name, uint64_t n, uint64_t in_align = 256) {
    Shape s{};
    s.name = name;
    s.n = n;
    s.C = (n + 4095) / 4096 * 1024;  // calc_padding_len with k = 4
    s.cols = s.C / 1024;
    s.N = 8 * s.cols;
    s.bpo = (s.cols + 7) / 8;
    s.in_stride = (n + in_align - 1) / in_align * in_align;
    s.out_stride = (8 + 8 * s.C + 64 * (s.N - 1) + 255) / 256 * 256;
    std::vector<uint64_t> coff(s.N);
    for (uint64_t i = 0; i < s.N; ++i) coff[i] = bao::chunk_stream_off(i, s.N);
    CK(hipMalloc(&s.coff, s.N * 8));
    CK(hipMemcpy(s.coff, coff.data(), s.N * 8, hipMemcpyHostToDevice));
    return s;
}

struct Variant {
    const char *label;
    void (*fn)(fused::FusedArgs);
    int shape;  // 0: 16 MiB, 1: level-15 shape, 2: level-15 shape with 16-B row stride, 3: 16 MiB rows + 16 B
    bool full;
};

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 256;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    Shape sh[4] = {make_shape("16MiB", 16ull << 20), make_shape("L15 (16779371 B)", 16779371ull),
                   make_shape("L15, 16-B row stride", 16779371ull, 16), make_shape("16MiB", 16ull << 20, 256)};
    sh[3].in_stride = (16ull << 20) + 16;
    sh[3].name = "16MiB, rows 16 MiB + 16 B";
    const uint64_t in_bytes = count * sh[1].in_stride, out_bytes = count * sh[1].out_stride;
    uint8_t *in, *out, *cv;
    CK(hbm::Allocator::get().alloc(in_bytes, reinterpret_cast<void **>(&in)));
    CK(hbm::Allocator::get().alloc(out_bytes, reinterpret_cast<void **>(&out)));
    const uint64_t cv_bytes = count * 8 * (8 * sh[1].bpo) * 32;  // >= count * N * 32 for both shapes
    CK(hipMalloc(&cv, cv_bytes));
    uint8_t *cv3;  // run mode: level-3 CVs
    CK(hipMalloc(&cv3, count * sh[1].N / 8 * 32));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, in_bytes / 8, 0xCA4B0AD0ull);
    CK(hipMemset(out, 0, out_bytes));
    std::vector<uint8_t> enc = zfec_enc_matrix(4, 8);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(4 * 256, 0);
    for (int s = 0; s < 4; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < 4; ++r) tab[s * 256 + x] |= (uint32_t)gf.mul(enc[(4 + r) * 4 + s], (uint8_t)x) << (8 * r);
    uint32_t *dtab, *dq;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dq, 4096));
    CK(hipMemset(dq, 0, 4096));
    using fused::zfec_bao_fused_kernel;
    // the product's template arguments (fused_kernels.hip KF32 / KG32), DG varied
    const std::vector<Variant> vs = {
        {"FULL product @16MiB", zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 0, true},
        {"general product @16MiB", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 0, false},
        {"general product @L15", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG13 no level-0 CV stores @L15", zfec_bao_fused_kernel<true, false, 1, 13, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG14 block-padded CV layout @L15", zfec_bao_fused_kernel<true, false, 1, 14, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG12 node slots zero-filled @L15", zfec_bao_fused_kernel<true, false, 1, 12, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG5 aligned lines @L15", zfec_bao_fused_kernel<true, false, 1, 5, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG1 no line stores @L15", zfec_bao_fused_kernel<true, false, 1, 1, 0, true, 1, 0, true, 1>, 1, false},
        {"general DG3 no GF @L15", zfec_bao_fused_kernel<true, false, 1, 3, 0, true, 1, 0, true, 1>, 1, false},
        {"FULL DG11 no tree node stores @16MiB", zfec_bao_fused_kernel<true, true, 1, 11, 0, true, 0, 0, true, 1>, 0, true},
        {"general DG13 no level-0 CV stores @16MiB", zfec_bao_fused_kernel<true, false, 1, 13, 0, true, 1, 0, true, 1>, 0, false},
        {"general DG14 block-padded CV layout @16MiB", zfec_bao_fused_kernel<true, false, 1, 14, 0, true, 1, 0, true, 1>, 0, false},
        {"general product @L15 16-B rows", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 2, false},
        {"FULL product @16MiB+16 rows", zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 3, true},
        {"FULL product @16MiB (again)", zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 0, true},
        {"general product @L15 (again)", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 1, false},
        {"general RT16 MP0 @L15 (run mode)", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 0, 0, true, 1, 8, false, 0, 16>, 1, false},
        {"general RT16 MP1 @L15", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1, 8, false, 0, 16>, 1, false},
        {"general RT8 MP0 @L15", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 0, 0, true, 1, 8, false, 0, 8>, 1, false},
        {"general RT32 MP0 @L15", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 0, 0, true, 1, 8, false, 0, 32>, 1, false},
        {"general product @L15 (third)", zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 1, false},
    };
    for (const auto &v : vs)
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(v.fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)fused::LDS_BYTES));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    printf("objects %llu, %d timed launches per variant after 1 warm-up; dispatch order below\n",
           (unsigned long long)count, reps);
    for (const auto &v : vs) {
        const Shape &s = sh[v.shape];
        fused::FusedArgs a{};
        a.in = in; a.in_stride = s.in_stride; a.valid = s.n; a.C = s.C;
        a.out = out; a.out_stride = s.out_stride;
        a.count = count; a.N = s.N; a.cols = s.cols; a.bpo = s.bpo;
        a.table = dtab; a.coff = s.coff; a.cv = cv; a.queue = dq; a.cvs = s.N / 8;
        a.cv3 = cv3;
        if (v.full && (s.cols % 8 || s.n < 4 * s.C)) { fprintf(stderr, "FULL needs cols %% 8 == 0\n"); return 1; }
        const uint64_t blocks = count * s.bpo;
        const unsigned grid = (unsigned)std::min<uint64_t>(256, (blocks + fused::FW - 1) / fused::FW);
        std::vector<float> ms;
        for (int r = 0; r <= reps; ++r) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(v.fn, dim3(grid), dim3(fused::FTPB), fused::LDS_BYTES, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double m = ms[ms.size() / 2];
        printf("VARIANT %-44s dispatches %d  median %7.3f ms  %7.1f GiB/s input  (%s)\n", v.label, reps + 1, m,
               count * s.n / (m * 1e-3) / 1073741824.0, s.name);
        fflush(stdout);
    }
    return 0;
}
