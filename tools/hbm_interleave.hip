// hbm_interleave.hip — physical chunk placement for the zfec batch buffers.
// hbm_partition showed device memory falls into "classes" of >= 1 GiB:
// writes spread over two classes run at ~6.9 TB/s, inside one class at
// ~5.4.  Here: create 1 GiB physical chunks (hipMemCreate), classify them
// by pairwise write timing, then map them (hipMemMap) behind the input and
// output VA ranges in different orders and time the product's 4-of-8 kernel
// (zfec_device.hpp) on each mapping.  Calibration tool, not product.
//   hbm_interleave [chunks=100] [rounds=3]
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

constexpr uint64_t GiB = 1ull << 30;
constexpr uint64_t RUN = 256 << 10;

__global__ __launch_bounds__(256) void pair_write(uint8_t *a, uint8_t *b, uint64_t block) {
    const uint32_t x = xcc_id();
    const uint32_t g = gridDim.x / 8, w = blockIdx.x / 8;
    uint8_t *reg = (x < 4 ? a : b) + (x & 3) * (block / 4);
    const uint64_t runs = block / 4 / RUN;
    const u32x4 val = {blockIdx.x, threadIdx.x, 1u, 2u};
    for (uint64_t r = w; r < runs; r += g) {
        uint8_t *p = reg + r * RUN + threadIdx.x * 16;
#pragma unroll 4
        for (int i = 0; i < (int)(RUN / 4096); ++i) __builtin_nontemporal_store(val, reinterpret_cast<u32x4 *>(p + i * 4096));
    }
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
    int bpc, chunk;
};

template <int U, int MAP, int CH, int WPE>
Variant V(int bpc) {
    char buf[64];
    snprintf(buf, sizeof buf, "U%d MAP%d CH%-3d bpc%d", U, MAP, CH, bpc);
    return Variant{buf, gf_apply_kernel<4, 1, U, MAP, true, 0, WPE, 0, true>, bpc, CH};
}

int main(int argc, char **argv) {
    const int nch = argc > 1 ? atoi(argv[1]) : 100;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    int dev = 0;
    CK(hipSetDevice(dev));
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    printf("allocation granularity %zu\n", gran);
    std::vector<hipMemGenericAllocationHandle_t> h(nch);
    for (int i = 0; i < nch; ++i) CK(hipMemCreate(&h[i], GiB, &prop, 0));
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    auto map_range = [&](uint8_t *va, const std::vector<int> &ids) {
        for (size_t i = 0; i < ids.size(); ++i) CK(hipMemMap(va + i * GiB, GiB, 0, h[ids[i]], 0));
        CK(hipMemSetAccess(va, ids.size() * GiB, &acc, 1));
    };
    auto unmap_range = [&](uint8_t *va, size_t n) { CK(hipMemUnmap(va, n * GiB)); };

    // ---- classify: map all chunks in creation order ----
    uint8_t *all = nullptr;
    CK(hipMemAddressReserve(reinterpret_cast<void **>(&all), (size_t)nch * GiB, GiB, nullptr, 0));
    std::vector<int> ids(nch);
    for (int i = 0; i < nch; ++i) ids[i] = i;
    map_range(all, ids);
    CK(hipMemset(all, 0, (size_t)nch * GiB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto rate = [&](int a, int b) {
        float best = 1e9f;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(pair_write, dim3(512), dim3(256), 0, 0, all + (size_t)a * GiB, all + (size_t)b * GiB, GiB);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            best = std::min(best, t);
        }
        return 2.0 * GiB / (best * 1e-3) / 1e9;
    };
    std::vector<int> reps, cls(nch, -1);
    std::vector<double> self;
    for (int i = 0; i < nch; ++i) {
        for (size_t r = 0; r < reps.size() && cls[i] < 0; ++r)
            if (rate(reps[r], i) < 1.12 * self[r]) cls[i] = (int)r;
        if (cls[i] < 0) {
            cls[i] = (int)reps.size();
            reps.push_back(i);
            self.push_back(rate(i, i));
        }
    }
    printf("classes: %zu (self rates:", reps.size());
    for (double s : self) printf(" %.0f", s);
    printf(")\nchunk classes: ");
    for (int i = 0; i < nch; ++i) printf("%d", cls[i]);
    printf("\n");
    unmap_range(all, nch);

    // ---- mappings for 1024 x 16 MiB: input 16 chunks, output 32 chunks ----
    const int K = 4, M = 8;
    const uint64_t n = 16ull << 20, C = n / K, count = 1024;
    std::vector<std::vector<int>> bycls(reps.size());
    for (int i = 0; i < nch; ++i) bycls[cls[i]].push_back(i);
    struct Mapping { std::string name; std::vector<int> in, out; };
    std::vector<Mapping> maps;
    {
        Mapping m{"creation order", {}, {}};
        for (int i = 0; i < 16; ++i) m.in.push_back(i);
        for (int i = 16; i < 48; ++i) m.out.push_back(i);
        maps.push_back(m);
    }
    auto take_rr = [&](int cnt, std::vector<size_t> &pos, const std::vector<int> &order) {
        std::vector<int> r;
        size_t k = 0;
        while ((int)r.size() < cnt) {
            const int c = order[k++ % order.size()];
            if (pos[c] < bycls[c].size()) r.push_back(bycls[c][pos[c]++]);
            if (k > 100000) break;
        }
        return r;
    };
    std::vector<int> all_cls;
    for (size_t c = 0; c < reps.size(); ++c) all_cls.push_back((int)c);
    // largest class first
    std::vector<int> by_size = all_cls;
    std::sort(by_size.begin(), by_size.end(), [&](int a, int b) { return bycls[a].size() > bycls[b].size(); });
    if (reps.size() >= 2) {
        std::vector<size_t> pos(reps.size(), 0);
        Mapping m{"interleaved (all classes round robin)", {}, {}};
        m.in = take_rr(16, pos, all_cls);
        m.out = take_rr(32, pos, all_cls);
        maps.push_back(m);
        std::vector<size_t> p2(reps.size(), 0);
        Mapping s{"one class as far as possible", {}, {}};
        s.in = take_rr(16, p2, by_size);  // round robin over a one-element order = one class
        std::vector<int> only{by_size[0]};
        std::vector<size_t> p3(reps.size(), 0);
        s.in = take_rr(std::min<int>(16, (int)bycls[by_size[0]].size()), p3, only);
        s.out = take_rr(std::min<int>(32, (int)bycls[by_size[0]].size() - (int)s.in.size()), p3, only);
        if (s.in.size() == 16 && s.out.size() == 32) maps.push_back(s);
        else printf("(largest class has %zu chunks: no one-class mapping)\n", bycls[by_size[0]].size());
    }
    for (auto &m : maps) {
        printf("mapping '%s': in", m.name.c_str());
        for (int i : m.in) printf(" %d", cls[i]);
        printf(" | out");
        for (int i : m.out) printf(" %d", cls[i]);
        printf("\n");
    }

    std::vector<uint8_t> enc = zfec_enc_matrix(K, M);
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> tab(K * 256, 0);
    for (int s = 0; s < K; ++s)
        for (int x = 0; x < 256; ++x)
            for (int r = 0; r < K; ++r)
                tab[s * 256 + x] |= (uint32_t)gf.mul(enc[(K + r) * K + s], (uint8_t)x) << (8 * r);
    uint32_t *dtab, *dq;
    CK(hipMalloc(&dtab, tab.size() * 4));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dq, 4096));
    CK(hipMemset(dq, 0, 4096));
    unsigned long long *dsum;
    CK(hipMalloc(&dsum, 8));
    std::vector<Variant> vs = {V<2, 3, 32, 2>(2), V<2, 6, 32, 2>(2), V<2, 6, 8, 2>(2), V<1, 6, 16, 1>(4)};
    uint8_t *in = nullptr, *out = nullptr;
    CK(hipMemAddressReserve(reinterpret_cast<void **>(&in), 16 * GiB, GiB, nullptr, 0));
    CK(hipMemAddressReserve(reinterpret_cast<void **>(&out), 32 * GiB, GiB, nullptr, 0));
    auto csum = [&](const uint8_t *p, uint64_t bytes) {
        CK(hipMemset(dsum, 0, 8));
        hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)p, bytes / 8, dsum);
        unsigned long long hs;
        CK(hipMemcpy(&hs, dsum, 8, hipMemcpyDeviceToHost));
        return hs;
    };
    {  // reference: plain hipMalloc buffers
        uint8_t *ri, *ro;
        CK(hipMalloc(&ri, count * n));
        CK(hipMalloc(&ro, count * 2 * n));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)ri, count * n / 8, 0xCA4B0AD0ull);
        ApplyArgs a{};
        a.in = ri; a.out = ro; a.in_stride = n; a.out_stride = M * C; a.valid = n; a.C = C;
        a.tiles_per_obj = C / TILE; a.total_tiles = a.tiles_per_obj * count; a.count = count;
        a.table = dtab; a.queue = dq; a.chunk = 32;
        for (int j = 0; j < ZF_MAXK; ++j) { a.in_off[j] = j < K ? j * C : 0; a.copy_off[j] = j < K ? j * C : NO_OUT; }
        for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < K ? (K + q) * C : NO_OUT;
        hipLaunchKernelGGL(vs[0].fn, dim3(512), dim3(TPB), 256 * 4 * 8 * 4, 0, a);
        printf("reference (hipMalloc): input %016llx output %016llx\n", csum(ri, count * n), csum(ro, count * 2 * n));
        CK(hipFree(ri));
        CK(hipFree(ro));
    }
    for (auto &m : maps) {
        map_range(in, m.in);
        map_range(out, m.out);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, count * n / 8, 0xCA4B0AD0ull);
        CK(hipMemset(out, 0, count * 2 * n));
        printf("mapping '%s': input checksum %016llx\n", m.name.c_str(), csum(in, count * n));
        ApplyArgs a{};
        a.in = in; a.out = out; a.in_stride = n; a.out_stride = M * C; a.valid = n; a.C = C;
        a.tiles_per_obj = C / TILE; a.total_tiles = a.tiles_per_obj * count; a.count = count;
        a.table = dtab; a.queue = dq;
        for (int j = 0; j < ZF_MAXK; ++j) { a.in_off[j] = j < K ? j * C : 0; a.copy_off[j] = j < K ? j * C : NO_OUT; }
        for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < K ? (K + q) * C : NO_OUT;
        std::vector<std::vector<float>> ms(vs.size());
        for (int rd = 0; rd < rounds; ++rd)
            for (size_t v = 0; v < vs.size(); ++v) {
                a.chunk = vs[v].chunk;
                hipLaunchKernelGGL(vs[v].fn, dim3(256 * vs[v].bpc), dim3(TPB), 256 * 4 * 8 * 4, 0, a);
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(vs[v].fn, dim3(256 * vs[v].bpc), dim3(TPB), 256 * 4 * 8 * 4, 0, a);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[v].push_back(t);
                if (rd == 0) printf("  %s output checksum %016llx\n", vs[v].name.c_str(), csum(out, count * 2 * n));
            }
        CK(hipMemset(dsum, 0, 8));
        hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)out, count * 2 * n / 8, dsum);
        unsigned long long hs;
        CK(hipMemcpy(&hs, dsum, 8, hipMemcpyDeviceToHost));
        printf("== mapping '%s' (output checksum %016llx)\n", m.name.c_str(), hs);
        for (size_t v = 0; v < vs.size(); ++v) {
            auto t = ms[v];
            std::sort(t.begin(), t.end());
            const double bytes = (double)count * 3 * n;
            printf("%-22s median %7.3f ms -> %7.1f GB/s (%.3f of 8 TB/s)  best %7.1f\n", vs[v].name.c_str(),
                   t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-3) / 1e9,
                   bytes / (t[t.size() / 2] * 1e-3) / 8e12, bytes / (t[0] * 1e-3) / 1e9);
        }
        CK(hipDeviceSynchronize());
        unmap_range(in, 16);
        unmap_range(out, 32);
    }
    return 0;
}
