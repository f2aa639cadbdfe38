// zfec_timeline.hip — where does the headline K1 launch lose time?  Runs the
// product's 4-of-8 kernel (carbonado_amd/csrc/zfec_device.hpp) with per-
// workgroup wall-clock traces (start, end, XCC, tiles) for the static
// XCD-grouped schedule (MAP 3) and the dynamic run queue (MAP 6/7),
// interleaved in one process, at 1024 and 2048 x 16 MiB.  Calibration tool,
// not product.
//   zfec_timeline [max_objects=2048] [rounds=5] [count:in_slot:out_slot:step ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../carbonado_amd/csrc/gf256.hpp"
#include "zfec_variants.hpp"

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
    int bpc, chunk, u;
    uint32_t mask = 0;
};

template <int U, int MAP, int CH, int WPE>
Variant V(int bpc) {
    char buf[96];
    snprintf(buf, sizeof buf, "U%d MAP%d CH%-3d bpc%d", U, MAP, CH, bpc);
    return Variant{buf, gf_apply_kernel<4, 1, U, MAP, true, 0, WPE, 0, true, false, true>, bpc, CH, U};
}

int main(int argc, char **argv) {
    const uint64_t maxc = argc > 1 ? atoll(argv[1]) : 2048;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int K = 4, M = 8;
    const uint64_t n = 16ull << 20, C = n / K;
    uint8_t *in, *out;
    CK(hipMalloc(&in, maxc * n));
    CK(hipMalloc(&out, maxc * 2 * n));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, maxc * n / 8, 0xCA4B0AD0ull);
    std::vector<uint8_t> enc = zfec_enc_matrix(K, M);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(K * 256, 0);
    for (int s = 0; s < K; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < K; ++r)
                tab[s * 256 + x] |= (uint32_t)gf.mul(enc[(K + r) * K + s], (uint8_t)x) << (8 * r);
    uint32_t *dtab, *dq;
    uint64_t *dtr;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dq, 4096));
    CK(hipMemset(dq, 0, 4096));
    CK(hipMalloc(&dtr, 1024 * 4 * 8));
    ApplyArgs a{};
    a.in = in; a.out = out; a.in_stride = n; a.out_stride = M * C; a.valid = n; a.C = C;
    a.tiles_per_obj = C / TILE; a.table = dtab; a.queue = dq; a.trace = dtr;
    for (int j = 0; j < ZF_MAXK; ++j) { a.in_off[j] = j < K ? j * C : 0; a.copy_off[j] = j < K ? j * C : NO_OUT; }
    for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < K ? (K + q) * C : NO_OUT;

    std::vector<Variant> vs = {V<2, 3, 32, 2>(2), V<2, 6, 32, 2>(2)};
    // ZT_MASKS=m1,m2,...: extra MAP 6 variants restricted to those XCD masks
    if (const char *e = getenv("ZT_MASKS")) {
        std::string ms(e);
        size_t p = 0;
        while (p < ms.size()) {
            size_t q = ms.find(',', p);
            if (q == std::string::npos) q = ms.size();
            Variant w = V<2, 6, 32, 2>(2);
            w.mask = (uint32_t)strtoul(ms.substr(p, q - p).c_str(), nullptr, 0);
            w.name += " xcd" + ms.substr(p, q - p);
            vs.push_back(w);
            p = q + 1;
        }
    }
    // layouts: {objects, first input slot, first output slot, slot stride in objects}; argv[3..] as c:i:o:s
    struct Layout { uint64_t count, first_in, first_out, step, step_out; };
    std::vector<Layout> layouts;
    for (int i = 3; i < argc; ++i) {
        unsigned long long c, fi, fo, st, so;
        const int nf = sscanf(argv[i], "%llu:%llu:%llu:%llu:%llu", &c, &fi, &fo, &st, &so);
        if (nf >= 4) layouts.push_back({c, fi, fo, st, nf == 5 ? so : st});
    }
    if (layouts.empty())
        layouts = {{1024, 0, 0, 1, 1}, {1024, 0, 0, maxc / 1024, maxc / 1024}, {maxc, 0, 0, 1, 1}};
    for (const Layout &ly : layouts)
        if (ly.count == 0 || ly.step == 0 || ly.first_in + (ly.count - 1) * ly.step >= maxc ||
            ly.step_out == 0 || ly.first_out + (ly.count - 1) * ly.step_out >= maxc) {
            fprintf(stderr, "layout out of range\n");
            return 1;
        }
    unsigned long long *dsum;
    CK(hipMalloc(&dsum, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Layout &ly : layouts) {
        const uint64_t count = ly.count;
        a.count = count;
        a.in = in + ly.first_in * n;
        a.out = out + ly.first_out * 2 * n;
        a.in_stride = ly.step * n;
        a.out_stride = ly.step_out * 2 * n;
        a.total_tiles = a.tiles_per_obj * count;
        std::vector<std::vector<float>> ms(vs.size());
        std::vector<std::vector<uint64_t>> last_tr(vs.size());
        unsigned long long ref = 0;
        for (int rd = 0; rd < rounds; ++rd) {
            for (size_t v = 0; v < vs.size(); ++v) {
                const int grid = 256 * vs[v].bpc;
                a.chunk = vs[v].chunk;
                a.xcd_mask = vs[v].mask;
                if (rd == 0) CK(hipMemset(out, 0, maxc * 2 * n));
                hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(TPB), 256 * 4 * 8 * 4, 0, a);  // warm
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(vs[v].fn, dim3(grid), dim3(TPB), 256 * 4 * 8 * 4, 0, a);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[v].push_back(t);
                last_tr[v].resize(grid * 4);
                CK(hipMemcpy(last_tr[v].data(), dtr, grid * 4 * 8, hipMemcpyDeviceToHost));
                if (rd == 0) {
                    CK(hipMemset(dsum, 0, 8));
                    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)out,
                                       maxc * 2 * n / 8, dsum);
                    unsigned long long h;
                    CK(hipMemcpy(&h, dsum, 8, hipMemcpyDeviceToHost));
                    if (v == 0) ref = h;
                    if (h != ref) printf("!! %s checksum mismatch\n", vs[v].name.c_str());
                }
            }
        }
        const double bytes = (double)count * 3 * n;
        printf("== %llu objects from input slot %llu, output slot %llu, every %llu / %llu\n", (unsigned long long)count,
               (unsigned long long)ly.first_in, (unsigned long long)ly.first_out, (unsigned long long)ly.step,
               (unsigned long long)ly.step_out);
        for (size_t v = 0; v < vs.size(); ++v) {
            auto t = ms[v];
            std::sort(t.begin(), t.end());
            // trace of the last launch: wall clock ticks of 10 ns
            const auto &tr = last_tr[v];
            const int G = (int)tr.size() / 4;
            uint64_t s0 = ~0ull, e_max = 0;
            for (int b = 0; b < G; ++b) { s0 = std::min(s0, tr[4 * b]); e_max = std::max(e_max, tr[4 * b + 1]); }
            std::vector<double> ends, starts;
            double xe[8] = {0}, xt[8] = {0}, xn[8] = {0};
            for (int b = 0; b < G; ++b) {
                const double e = (tr[4 * b + 1] - s0) * 1e-5, s = (tr[4 * b] - s0) * 1e-5;  // ms
                ends.push_back(e);
                starts.push_back(s);
                const int x = (int)tr[4 * b + 2] & 7;
                xe[x] = std::max(xe[x], e);
                xt[x] += (double)tr[4 * b + 3];
                xn[x] += 1;
            }
            std::sort(ends.begin(), ends.end());
            std::sort(starts.begin(), starts.end());
            printf("%-22s median %7.3f ms min %7.3f -> %7.1f GB/s (median) %7.1f (best) | span %.3f start p99 %.3f"
                   " end p1 %.3f p50 %.3f p99 %.3f\n",
                   vs[v].name.c_str(), t[t.size() / 2], t[0], bytes / (t[t.size() / 2] * 1e-3) / 1e9,
                   bytes / (t[0] * 1e-3) / 1e9, (e_max - s0) * 1e-5, starts[G * 99 / 100], ends[G / 100],
                   ends[G / 2], ends[G * 99 / 100]);
            printf("    per-XCC last end ms / tiles:");
            for (int x = 0; x < 8; ++x) printf(" %d:%.3f/%.0f(%.0fwg)", x, xe[x], xt[x], xn[x]);
            printf("\n");
        }
    }
    return 0;
}
