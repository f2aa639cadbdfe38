// fused_tune.hip — K13 (carbonado_amd/csrc/fused_device.hpp) variants and
// diagnostics on 256 x 16 MiB objects, interleaved in one process.  Times
// the fused kernel alone (the parent levels are not run).  Calibration tool.
//   fused_tune [objects=256] [rounds=3] [variant-name filter]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fused_variants.hpp"
#include "../carbonado_amd/csrc/gf256.hpp"
#include "../carbonado_amd/csrc/hbm_alloc.hpp"

using namespace chip;

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

// order-sensitive checksum of a buffer (the tuner compares every non-DG
// variant's stream and CVs with the first variant's)
__global__ void checksum_kernel(const uint64_t *p, size_t n, unsigned long long *out) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        acc += (p[i] ^ (i * 0x9E3779B97F4A7C15ull)) * ((i << 1) | 1);
    atomicAdd(out, acc);
}

static unsigned long long checksum(const uint8_t *p, size_t bytes) {
    unsigned long long *d, h = 0;
    CK(hipMalloc(&d, 8));
    CK(hipMemset(d, 0, 8));
    hipLaunchKernelGGL(checksum_kernel, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const uint64_t *>(p), bytes / 8, d);
    CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    return h;
}

struct Variant {
    std::string name;
    void (*fn)(fused::FusedArgs);
    int kind;  // 0: zfec 4-of-8 + bao of the shards, 1: bao of the content
    bool spec = false;  // K13S: 12-wave workgroups, roles on separate waves
};

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 256;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    const uint64_t n = 16ull << 20, C = n / 4;
    const uint64_t N0 = 8 * C / 1024, N1 = n / 1024;  // chunks per stream: KIND 0 (zfec output), KIND 1 (content)
    const uint64_t blen0 = 8 + 8 * C + 64 * (N0 - 1), bstride = (blen0 + 255) / 256 * 256;
    uint8_t *in, *out, *cv;
    CK(hbm::Allocator::get().alloc(count * n, reinterpret_cast<void **>(&in)));
    CK(hbm::Allocator::get().alloc(count * bstride + 256, reinterpret_cast<void **>(&out)));
    // FT_SOFF=56: every stream 56 B into its row (the library's layout since
    // round 5: each chunk and node on a 64-B boundary); 0: at the row start
    const uint64_t soff = getenv("FT_SOFF") ? (uint64_t)atoll(getenv("FT_SOFF")) & 248 : 0;
    printf("streams %llu B into their rows\n", (unsigned long long)soff);
    CK(hipMalloc(&cv, count * N0 * 32));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, count * n / 8, 0xCA4B0AD0ull);
    std::vector<uint8_t> enc = zfec_enc_matrix(4, 8);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(4 * 256, 0);
    for (int s = 0; s < 4; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < 4; ++r) tab[s * 256 + x] |= (uint32_t)gf.mul(enc[(4 + r) * 4 + s], (uint8_t)x) << (8 * r);
    uint32_t *dtab;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    uint64_t *dcoff[2];
    for (int k = 0; k < 2; ++k) {
        const uint64_t N = k ? N1 : N0;
        std::vector<uint64_t> coff(N);
        for (uint64_t i = 0; i < N; ++i) coff[i] = bao::chunk_stream_off(i, N);
        CK(hipMalloc(&dcoff[k], N * 8));
        CK(hipMemcpy(dcoff[k], coff.data(), N * 8, hipMemcpyHostToDevice));
    }
    uint32_t *dq;
    CK(hipMalloc(&dq, 4096));
    CK(hipMemset(dq, 0, 4096));
    fused::FusedArgs A[2];
    for (int k = 0; k < 2; ++k) {
        fused::FusedArgs &a = A[k];
        a = fused::FusedArgs{};
        a.in = in; a.in_stride = n; a.valid = n; a.C = k ? 0 : C; a.out = out + soff; a.out_stride = bstride;
        a.count = count; a.N = k ? N1 : N0; a.cols = k ? 0 : C / 1024; a.bpo = k ? N1 / 64 : (C / 1024 + 7) / 8;
        a.table = dtab; a.coff = dcoff[k]; a.cv = cv; a.queue = dq;
        a.cvs = a.N / 8;  // level-3 CVs per object (FULL)
    }
    const char *which = argc > 3 ? argv[3] : "all";
    std::vector<Variant> all = {
        {"K0 FULL (product)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 0},
        {"K0 FULL O32 GFP0", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 0>, 0},
        {"K0 FULL O32=0 GFP0 (r6 product)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0>, 0},
        {"K0 FULL K13S spec", fused::zfec_bao_spec_kernel<true>, 0, true},
        {"K0 FULL product PRIO1 (GF/stores at raised priority)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1, 8, false, 1>, 0},
        {"K1 product PRIO1 (loads/stores at raised priority)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 1, true, 0, 0, true, 0, 8, true, 1>, 1},
        {"K1 product NTL (as the library)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 1, true, 0, 0, true, 0, 8, true>, 1},
        {"K0 FULL product NTL (nontemporal loads)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1, 8, true>, 0},
        {"K0 FULL product WPG4 (1 wave/SIMD)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1, 4>, 0},
        {"K0 FULL K13S spec NPB1", fused::zfec_bao_spec_kernel<true, 1>, 0, true},
        {"K0 FULL MP1", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 1>, 0},
        {"K0 FULL ORD2 MP1", fused::zfec_bao_fused_kernel<true, true, 2, 0, 0, true, 1>, 0},
        {"K1 MP1", fused::zfec_bao_fused_kernel<true, true, 1, 0, 1, true, 1>, 1},
        {"K0 general MP1", fused::zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1>, 0},
        {"K0 general ORD2", fused::zfec_bao_fused_kernel<true, false, 2, 0, 0, true, 0>, 0},
        {"K0 general ORD2 MP1", fused::zfec_bao_fused_kernel<true, false, 2, 0, 0, true, 1>, 0},
        {"K0 FULL ORD2 NT0", fused::zfec_bao_fused_kernel<false, true, 2, 0, 0>, 0},
        {"K0 general ORD2 NT0", fused::zfec_bao_fused_kernel<false, false, 2, 0, 0>, 0},
        {"K0 FULL ORD0", fused::zfec_bao_fused_kernel<true, true, 0, 0, 0>, 0},
        {"K0 FULL ORD2", fused::zfec_bao_fused_kernel<true, true, 2, 0, 0>, 0},
        {"K0 FULL ORD3", fused::zfec_bao_fused_kernel<true, true, 3, 0, 0>, 0},
        {"K1 ORD2", fused::zfec_bao_fused_kernel<true, true, 2, 0, 1>, 1},
        {"K1 ORD3", fused::zfec_bao_fused_kernel<true, true, 3, 0, 1>, 1},
        {"K0 general", fused::zfec_bao_fused_kernel<true, false, 1, 0, 0>, 0},
        {"K1 (product)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 1>, 1},
        {"K0 DG1 no line stores/reads", fused::zfec_bao_fused_kernel<true, true, 1, 1, 0>, 0},
        {"K0 DG7 piece reads, no stores", fused::zfec_bao_fused_kernel<true, true, 1, 7, 0>, 0},
        {"K0 DG2 no hash", fused::zfec_bao_fused_kernel<true, true, 1, 2, 0>, 0},
        {"K0 DG8 line stores to L2", fused::zfec_bao_fused_kernel<true, true, 1, 8, 0>, 0},
        {"K0 FULL SS1", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 1>, 0},
        {"K0 FULL SS1 ORD2", fused::zfec_bao_fused_kernel<true, true, 2, 0, 0, true, 0, 1>, 0},
        {"K0 general SS1 MP1", fused::zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 1>, 0},
        {"K1 SS1", fused::zfec_bao_fused_kernel<true, true, 1, 0, 1, true, 0, 1>, 1},
        {"K0 DG8 ORD2 line stores to L2", fused::zfec_bao_fused_kernel<true, true, 2, 8, 0>, 0},
        {"K0 DG5 aligned lines", fused::zfec_bao_fused_kernel<true, true, 1, 5, 0>, 0},
        {"K1 DG5 aligned lines", fused::zfec_bao_fused_kernel<true, true, 1, 5, 1>, 1},
        {"K1 DG1 no line stores/reads", fused::zfec_bao_fused_kernel<true, true, 1, 1, 1>, 1},
        {"K1 DG7 piece reads, no stores", fused::zfec_bao_fused_kernel<true, true, 1, 7, 1>, 1},
        {"K1 DG2 no hash", fused::zfec_bao_fused_kernel<true, true, 1, 2, 1>, 1},
        {"K0 FULL K13S spec (again)", fused::zfec_bao_spec_kernel<true>, 0, true},
        {"K0 FULL (product, again)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 0},
        // round 4: occupancy and LDS-conflict diagnostics (wrong output)
        {"K0 DG10 GF lookups conflict-free", fused::zfec_bao_fused_kernel<true, true, 1, 10, 0, true, 0, 0, true, 1>, 0},
        {"K0 DG3 no GF (product params)", fused::zfec_bao_fused_kernel<true, true, 1, 3, 0, true, 0, 0, true, 1>, 0},
        {"K0 DG1 no line stores/reads (product params)", fused::zfec_bao_fused_kernel<true, true, 1, 1, 0, true, 0, 0, true, 1>, 0},
        {"K0 DG7 piece reads, no stores (product params)", fused::zfec_bao_fused_kernel<true, true, 1, 7, 0, true, 0, 0, true, 1>, 0},
        {"K0 DG-occ WPG12 3 waves/SIMD rows aliased", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1, 12>, 0},
        {"K0 general product", fused::zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1>, 0},
        {"K0 general DG-occ WPG12 3 waves/SIMD rows aliased", fused::zfec_bao_fused_kernel<true, false, 1, 0, 0, true, 1, 0, true, 1, 12>, 0},
        {"K0 FULL (product, third)", fused::zfec_bao_fused_kernel<true, true, 1, 0, 0, true, 0, 0, true, 1>, 0}};
    std::vector<Variant> vs;
    for (auto &v : all)
        if (!strcmp(which, "all") || strstr(v.name.c_str(), which)) vs.push_back(v);
    for (auto &v : vs)
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(v.fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(v.spec ? fused::S_LDS_BYTES : fused::LDS_BYTES));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(vs.size());
    std::vector<unsigned long long> sums(vs.size(), 0);
    for (int rd = 0; rd < rounds; ++rd)
        for (size_t v = 0; v < vs.size(); ++v) {
            const fused::FusedArgs &a = A[vs[v].kind];
            const uint64_t blocks = count * a.bpo;
            const unsigned grid = (unsigned)std::min<uint64_t>(256, (blocks + fused::FW - 1) / fused::FW);
            const unsigned tpb = vs[v].spec ? (vs[v].name.find("NPB1") != std::string::npos ? fused::stpb<1>() : fused::STPB)
                                 : vs[v].name.find("WPG4") != std::string::npos ? 256u
                                 : vs[v].name.find("WPG12") != std::string::npos ? 768u : fused::FTPB;
            const size_t ldsb = vs[v].spec ? fused::S_LDS_BYTES : fused::LDS_BYTES;
            hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(tpb), ldsb, 0, a);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(tpb), ldsb, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t);
            if (rd == 0) {  // output of this variant: streams + CVs
                CK(hipMemset(out, 0, count * bstride));
                CK(hipMemset(cv, 0, count * N0 * 32));
                hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(tpb), ldsb, 0, a);
                CK(hipDeviceSynchronize());
                sums[v] = checksum(out, count * bstride) ^ (checksum(cv, count * N0 * 32) * 3);
            }
        }
    {  // levels 1-3 from level-0 CVs (what the general path adds): bao_levels123_kernel, node-store variants
        const uint64_t N = N0, n3 = N / 8, work = count * n3;
        uint8_t *cv3;
        CK(hipMalloc(&cv3, count * n3 * 32));
        void (*kv[5])(const uint8_t *, uint64_t, uint64_t, const uint64_t *, uint8_t *, uint64_t, uint8_t *, uint64_t) = {
            fused::bao_levels123_kernel<1>, fused::bao_levels123_kernel<2>, fused::bao_levels123_kernel<0>, nullptr,
            fused::bao_levels123_seg_kernel};
        void (*kq[8])(const uint8_t *, uint64_t, uint64_t, const uint64_t *, uint8_t *, uint64_t, uint8_t *, uint64_t,
                      uint64_t, uint64_t, uint64_t) = {nullptr, nullptr, nullptr, fused::bao_levels123_lds_kernel<4>,
                                                       nullptr, fused::bao_levels123_lds_kernel<1>,
                                                       fused::bao_levels123_lds_kernel<2>,
                                                       fused::bao_levels123_lds_kernel<4>};
        const char *kn[8] = {"8-B node stores", "16-B node stores", "no node stores (diagnostic)",
                             "LDS-staged node stores, a level per round (QS 4, product)",
                             "node stacks as whole 64-B segments (SEG)",
                             "LDS-staged node stores, a node per round (QS 1)",
                             "LDS-staged node stores, two nodes per round (QS 2)",
                             "QS 4, stream base shifted 56 B: every node 64-B aligned (diagnostic, wrong bytes)"};
        std::vector<float> t3[8];
        unsigned long long sum3[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int rd = 0; rd < rounds + 1; ++rd)
            for (int k = 0; k < 8; ++k) {
                const int tpb = (k == 3 || k >= 5) ? 64 : 256;
                CK(hipEventRecord(e0));
                if (kq[k])
                    hipLaunchKernelGGL(kq[k], dim3((unsigned)((work + tpb - 1) / tpb)), dim3(tpb), 0, 0, cv, N, count,
                                       dcoff[0], out + (k == 7 ? 56 : 0), bstride, cv3, n3, (uint64_t)0,
                                       (uint64_t)0, (uint64_t)0);
                else
                    hipLaunchKernelGGL(kv[k], dim3((unsigned)((work + tpb - 1) / tpb)), dim3(tpb), 0, 0, cv, N, count,
                                       dcoff[0], out, bstride, cv3, n3);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (rd) t3[k].push_back(t);
                if (rd == 0) sum3[k] = checksum(out, count * bstride) ^ (checksum(cv3, count * n3 * 32) * 3);
            }
        printf("levels 1-3 outputs: LDS-staged %s 8-B stores; 16-B %s; SEG %s; QS 1 %s; QS 2 %s\n",
               sum3[3] == sum3[0] ? "==" : "!=", sum3[1] == sum3[0] ? "==" : "!=", sum3[4] == sum3[0] ? "==" : "!=",
               sum3[5] == sum3[0] ? "==" : "!=", sum3[6] == sum3[0] ? "==" : "!=");
        for (int k = 0; k < 8; ++k) {
            std::sort(t3[k].begin(), t3[k].end());
            printf("levels 1-3 from chunk CVs (bao_levels123_kernel), %s, %llu objects: median %.3f ms\n", kn[k],
                   (unsigned long long)count, t3[k][t3[k].size() / 2]);
        }
        CK(hipFree(cv3));
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto t = ms[v];
        std::sort(t.begin(), t.end());
        const double m = t[t.size() / 2];
        // 672 lane-ops per compression, 16 per chunk
        const double ops = (double)count * A[vs[v].kind].N * 16 * 672;
        const bool diag = vs[v].name.find("DG") != std::string::npos;
        size_t ref = 0;
        auto general = [&](size_t i) { return vs[i].name.find("general") != std::string::npos; };
        while (ref < vs.size() && (vs[ref].kind != vs[v].kind || general(ref) != general(v) ||
                                   vs[ref].name.find("DG") != std::string::npos))
            ++ref;
        const char *chk = diag ? "(diagnostic)" : (ref < vs.size() && sums[ref] == sums[v] ? "output = first" : "OUTPUT DIFFERS");
        printf("%-16s ", chk);
        printf("%-26s median %7.3f ms  -> %6.1f GiB/s input, %.3f of VALU (chunk compressions only)\n",
               vs[v].name.c_str(), m, count * n / (m * 1e-3) / 1073741824.0, ops / (m * 1e-3) / 39.3e12);
    }
    return 0;
}
