// zfec_tune.hip — sweep schedule variants of the product's K1 kernel
// (carbonado_amd/csrc/zfec_device.hpp) on the cfg2 workload, interleaved in
// one process (cdna_hip_programming.md rule 24).  Calibration tool, not product.
//   zfec_tune [objects=1024] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../carbonado_amd/csrc/gf256.hpp"
#include "zfec_variants.hpp"
#include "bao_variants.hpp"

using namespace chip;
using namespace chip::zf;

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
            exit(1);                                                                          \
        }                                                                                     \
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

__global__ void checksum_kernel(const uint64_t *p, size_t n, unsigned long long *out) {
    uint64_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        acc += p[i] * (2 * i + 1);
    atomicAdd(out, (unsigned long long)acc);
}

struct Variant {
    std::string name;
    void (*fn)(ApplyArgs);
    int blocks_per_cu;
    int chunk;
    size_t lds;
    bool bl = false;
};

template <int U, int MAP, bool NT, int CH = 1, int WPE = 1, int SB = 0, bool PF = false, bool NTL = false>
Variant V(int bpc) {
    char buf[96];
    snprintf(buf, sizeof buf, "U%d MAP%d CH%-3d wpe%d sb%d pf%d ntl%d %s bpc%d", U, MAP, CH, WPE, SB, PF, NTL,
             NT ? "nt " : "pln", bpc);
    return Variant{buf, gf_apply_kernel<4, 1, U, MAP, NT, 0, WPE, SB, PF, NTL>, bpc, CH, (size_t)256 * 4 * 8 * 4};
}

// bao-layout kernel (encode() Zfec|Bao): chunk slots of a bao stream, wave runs of CH 1 KiB units
template <bool NT, int CH, bool BL = true>
Variant VBL(int bpc) {
    char buf[96];
    snprintf(buf, sizeof buf, "%s wave-runs CH%-3d %s bpc%d", BL ? "BAO-LAYOUT" : "shard-major", CH, NT ? "nt " : "pln",
             bpc);
    return Variant{buf, gf_apply_bl_kernel<NT, BL>, bpc, CH, (size_t)256 * 4 * 8 * 4, BL};
}

// 8-of-16 variants (K = 8, NG = 2), replica count R
template <int U, int MAP, bool NT, int R, int CH = 1, int WPE = 1, int SB = 0, bool PF = false>
Variant V16(int bpc) {
    char buf[80];
    snprintf(buf, sizeof buf, "8of16 U%d MAP%d CH%-3d R%d wpe%d sb%d pf%d %s bpc%d", U, MAP, CH, R, WPE, SB, PF, NT ? "nt " : "pln", bpc);
    return Variant{buf, gf_apply_kernel<8, 2, U, MAP, NT, R, WPE, SB, PF>, bpc, CH, (size_t)256 * 8 * R * 8};
}

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int shape = argc > 3 ? atoi(argv[3]) : 4;  // 4 = 4-of-8, 8 = 8-of-16
    const int K = shape == 8 ? 8 : 4, M = 2 * K;
    const uint64_t n = 16ull << 20, C = n / K;
    uint8_t *in, *out;
    // ZT_CONTIG=1: physically contiguous device allocations (hipDeviceMallocContiguous)
    const bool contig = getenv("ZT_CONTIG") && atoi(getenv("ZT_CONTIG"));
    auto dmalloc = [&](uint8_t **p, size_t bytes) {
        if (contig) CK(hipExtMallocWithFlags(reinterpret_cast<void **>(p), bytes, hipDeviceMallocContiguous));
        else CK(hipMalloc(p, bytes));
    };
    dmalloc(&in, count * n);
    // bao layout variants write a whole bao stream per object (8 + 2n + 64 (N - 1) bytes)
    const uint64_t Nch = 2 * n / 1024;
    const uint64_t blen = 8 + 2 * n + 64 * (Nch - 1), bstride = (blen + 255) / 256 * 256;
    dmalloc(&out, count * (bstride > 2 * n ? bstride : 2 * n));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, count * n / 8, 0xCA4B0AD0ull);
    CK(hipMemset(out, 0, count * 2 * n));

    // packed parity table [s][x] of NG dwords
    const int NG = K / 4;
    std::vector<uint8_t> enc = zfec_enc_matrix(K, M);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(K * 256 * NG, 0);
    for (int s = 0; s < K; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < K; ++r)
                tab[(s * 256 + x) * NG + r / 4] |= (uint32_t)gf.mul(enc[(K + r) * K + s], (uint8_t)x) << (8 * (r % 4));
    uint32_t *dtab;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));

    std::vector<uint64_t> boff(Nch);
    for (uint64_t i = 0; i < Nch; ++i) boff[i] = chip::bao::chunk_stream_off(i, Nch);
    uint64_t *dboff;
    CK(hipMalloc(&dboff, Nch * 8));
    CK(hipMemcpy(dboff, boff.data(), Nch * 8, hipMemcpyHostToDevice));
    ApplyArgs a{};
    a.in = in; a.out = out; a.in_stride = n; a.out_stride = 2 * n; a.valid = n; a.C = C;
    a.tiles_per_obj = C / TILE; a.total_tiles = a.tiles_per_obj * count; a.count = count;
    a.out_stride = M * C;
    a.table = dtab;
    for (int j = 0; j < ZF_MAXK; ++j) { a.in_off[j] = j < K ? j * C : 0; a.copy_off[j] = j < K ? j * C : NO_OUT; }
    for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < K ? (K + q) * C : NO_OUT;

    std::vector<Variant> vs;
    if (K == 4)
        vs = {V<2, 3, true, 32, 2, 0, true>(2),  V<1, 3, true, 64, 1, 0, true>(4),  V<2, 3, true, 32, 2, 0, true>(1),
              V<2, 3, false, 32, 2, 0, true>(2), V<1, 3, false, 64, 1, 0, true>(4), V<2, 3, false, 32, 2, 0, true>(1),
              V<2, 3, true, 16, 2, 0, true>(1),  V<2, 3, true, 64, 2, 0, true>(1)};
    else
        vs = {V16<1, 3, true, 4, 64>(1),                V16<1, 3, true, 4, 64, 2, 1, true>(2),
              V16<1, 3, true, 4, 64, 2, 1, true>(1),    V16<1, 3, true, 4, 64, 1, 0, true>(1),
              V16<1, 3, true, 4, 64, 2, 2, true>(2),    V16<1, 3, true, 4, 16, 2, 1, true>(2),
              V16<1, 3, true, 4, 64, 3, 1>(2),          V16<1, 3, false, 4, 64, 2, 1, true>(2),
              V16<1, 3, false, 4, 64, 2, 1, true>(1),   V16<1, 3, false, 4, 32, 2, 1, true>(2)};
    unsigned long long *dsum;
    CK(hipMalloc(&dsum, 8));
    std::vector<std::vector<float>> ms(vs.size());
    unsigned long long ref = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rd = 0; rd < rounds; ++rd) {
        for (size_t v = 0; v < vs.size(); ++v) {
            const int grid = 256 * vs[v].blocks_per_cu;
            a.chunk = vs[v].chunk;
            a.bao_off = vs[v].bl ? dboff : nullptr;
            a.tiles_per_obj = C / TILE;
            a.bao_n = Nch;
            a.out_stride = vs[v].bl ? bstride : M * C;
            if (rd == 0) CK(hipMemset(out, 0, count * 2 * n));  // a variant that skips bytes fails the checksum
            if (rd == 0 && vs[v].bl) CK(hipMemset(out, 0, count * bstride));
            hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(TPB), vs[v].lds, 0, a);  // warm
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(TPB), vs[v].lds, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t);
            if (rd == 0) {
                CK(hipMemset(dsum, 0, 8));
                hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)out,
                                   count * 2 * n / 8, dsum);
                unsigned long long h;
                CK(hipMemcpy(&h, dsum, 8, hipMemcpyDeviceToHost));
                if (v == 0) ref = h;
                if (!vs[v].bl && h != ref) printf("!! %s checksum mismatch\n", vs[v].name.c_str());
            }
        }
    }
    const double bytes = (double)count * 3 * n;
    for (size_t v = 0; v < vs.size(); ++v) {
        auto t = ms[v];
        std::sort(t.begin(), t.end());
        printf("%-22s median %7.3f ms  min %7.3f ms  -> %7.1f GB/s (median)  %7.1f (best)\n", vs[v].name.c_str(),
               t[t.size() / 2], t[0], bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / (t[0] * 1e-3) / 1e9);
    }
    return 0;
}
