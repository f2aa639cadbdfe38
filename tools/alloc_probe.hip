// alloc_probe.hip — the same 1024 x 16 MiB 4-of-8 encode (zfec_device.hpp)
// on batch buffers from different allocators: hipMalloc, the contiguous
// allocator, and buffers built from hipMemCreate chunks of 256 MiB / 1 GiB /
// 4 GiB mapped once, in creation order, behind one fresh VA range.  Every
// mapping is made once and never remapped (a VA range re-mapped to other
// chunks read stale translations in hbm_interleave).  Calibration tool.
//   alloc_probe [rounds=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <cstdlib>
#include <string>
#include <vector>

#include "../carbonado_amd/csrc/gf256.hpp"
#include "zfec_variants.hpp"
#include "../carbonado_amd/csrc/hbm_alloc.hpp"

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

struct Buf {
    uint8_t *p = nullptr;
    std::vector<hipMemGenericAllocationHandle_t> h;
    uint64_t bytes = 0, chunk = 0;
    int kind = 0;  // 0 hipMalloc, 1 contiguous, 2 chunked, 3 class-balanced (hbm_alloc.hpp)
};

// VMM buffers are carved from one VA arena reserved at start and never
// reused: a VA range that had been mapped before (by hipMalloc or with other
// chunk sizes) read stale translations when re-mapped (outputs mismatched).
uint8_t *g_arena = nullptr;
uint64_t g_arena_used = 0, g_arena_size = 0;

uint64_t g_last_off = 0;
void meminfo(const char *what) {
    size_t fr = 0, tot = 0;
    CK(hipMemGetInfo(&fr, &tot));
    printf("  [%s] free %.1f GiB of %.1f\n", what, fr / 1073741824.0, tot / 1073741824.0);
}

Buf make(int kind, uint64_t bytes, uint64_t chunk, bool shuffle = false, bool reuse = false) {
    Buf b;
    b.kind = kind;
    b.bytes = bytes;
    b.chunk = chunk;
    if (kind == 3) {
        CK(chip::hbm::Allocator::get().alloc(bytes, reinterpret_cast<void **>(&b.p)));
        chip::hbm::Allocation A;
        chip::hbm::Allocator::get().info(b.p, &A);
        printf("  balanced: %llu groups made, classes found %u used %u, %.3f s\n", (unsigned long long)A.groups_made,
               A.classes_found, A.classes_used, A.seconds);
    } else if (kind == 0) CK(hipMalloc(&b.p, bytes));
    else if (kind == 1) CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&b.p), bytes, hipDeviceMallocContiguous));
    else {
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        const uint64_t al = 1ull << 30;
        g_arena_used = (g_arena_used + al - 1) / al * al;
        if (g_arena_used + bytes > g_arena_size) { fprintf(stderr, "arena exhausted\n"); exit(1); }
        if (reuse) {  // the range the previous chunked buffer of this size used
            b.p = g_arena + g_last_off;
            g_last_off += bytes;
        } else {
            b.p = g_arena + g_arena_used;
            g_last_off = g_arena_used;
            g_arena_used += bytes;
        }
        for (uint64_t o = 0; o < bytes; o += chunk) {
            hipMemGenericAllocationHandle_t h;
            CK(hipMemCreate(&h, chunk, &prop, 0));
            b.h.push_back(h);
        }
        std::vector<hipMemGenericAllocationHandle_t> order = b.h;
        if (shuffle) std::shuffle(order.begin(), order.end(), std::mt19937_64(42));
        for (size_t i = 0; i < order.size(); ++i) CK(hipMemMap(b.p + i * chunk, chunk, 0, order[i], 0));
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess(b.p, bytes, &acc, 1));
    }
    return b;
}

// frees the memory; the VA range is never reused
void drop(Buf &b) {
    CK(hipDeviceSynchronize());
    if (b.kind == 3) chip::hbm::Allocator::get().free(b.p);
    else if (b.kind < 2) CK(hipFree(b.p));
    else {
        for (uint64_t o = 0; o < b.bytes; o += b.chunk) CK(hipMemUnmap(b.p + o, b.chunk));  // one mapping at a time
        for (auto h : b.h) CK(hipMemRelease(h));
        // the VA stays reserved (arena): never mapped again
    }
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    g_arena_size = 4ull << 40;  // 4 TiB of VA
    CK(hipMemAddressReserve(reinterpret_cast<void **>(&g_arena), g_arena_size, 1ull << 30, nullptr, 0));
    printf("VA arena at %p\n", (void *)g_arena);
    const int K = 4, M = 8;
    const uint64_t n = 16ull << 20, C = n / K, count = 1024;
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
    auto csum = [&](const uint8_t *p, uint64_t bytes) {
        CK(hipMemset(dsum, 0, 8));
        hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)p, bytes / 8, dsum);
        unsigned long long hs;
        CK(hipMemcpy(&hs, dsum, 8, hipMemcpyDeviceToHost));
        return hs;
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<Variant> vs = {V<2, 3, 32, 2>(2), V<2, 6, 32, 2>(2), V<2, 7, 32, 2>(2), V<1, 6, 16, 1>(4)};
    struct Alloc { std::string name; int kind; uint64_t chunk; bool shuffle; bool reuse = false; };
    const uint64_t MiB = 1ull << 20;
    std::vector<Alloc> allocs = {{"balanced", 3, 0, false},
                                 {"hipMalloc", 0, 0, false},
                                 {"balanced (again)", 3, 0, false},
                                 {"hipMalloc (again)", 0, 0, false},
                                 {"balanced (3rd)", 3, 0, false}};
    unsigned long long ref = 0;
    for (size_t ai = 0; ai < allocs.size(); ++ai) {
        const Alloc &al = allocs[ai];
        const auto t0 = std::chrono::steady_clock::now();
        if (al.reuse) g_last_off = g_last_off - count * n;  // back to the previous pair's input range
        Buf bi = make(al.kind, count * n, al.chunk, al.shuffle, al.reuse);
        if (!al.reuse) g_arena_used = (g_arena_used + (1ull << 30) - 1) / (1ull << 30) * (1ull << 30);
        Buf bo = make(al.kind, count * 2 * n, al.chunk, al.shuffle, al.reuse);
        meminfo("allocated");
        CK(hipDeviceSynchronize());
        const double alloc_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)bi.p, count * n / 8, 0xCA4B0AD0ull);
        CK(hipMemset(bo.p, 0, count * 2 * n));
        ApplyArgs a{};
        a.in = bi.p; a.out = bo.p; a.in_stride = n; a.out_stride = M * C; a.valid = n; a.C = C;
        a.tiles_per_obj = C / TILE; a.total_tiles = a.tiles_per_obj * count; a.count = count;
        a.table = dtab; a.queue = dq;
        for (int j = 0; j < ZF_MAXK; ++j) { a.in_off[j] = j < K ? j * C : 0; a.copy_off[j] = j < K ? j * C : NO_OUT; }
        for (int q = 0; q < ZF_MAXP; ++q) a.par_off[q] = q < K ? (K + q) * C : NO_OUT;
        std::vector<std::vector<float>> ms(vs.size());
        bool ok = true;
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
                if (rd == 0) {
                    const unsigned long long h = csum(bo.p, count * 2 * n);
                    if (ai == 0 && v == 0) ref = h;
                    if (h != ref) ok = false;
                    CK(hipMemset(bo.p, 0, count * 2 * n));
                }
            }
        printf("== %s: in %p out %p, allocated in %.3f s, outputs %s\n", al.name.c_str(), (void *)bi.p, (void *)bo.p,
               alloc_s, ok ? "match" : "MISMATCH");
        for (size_t v = 0; v < vs.size(); ++v) {
            auto t = ms[v];
            std::sort(t.begin(), t.end());
            const double bytes = (double)count * 3 * n;
            printf("%-22s median %7.3f ms -> %7.1f GB/s (%.3f of 8 TB/s)  best %7.1f\n", vs[v].name.c_str(),
                   t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / (t[t.size() / 2] * 1e-3) / 8e12,
                   bytes / (t[0] * 1e-3) / 1e9);
        }
        fflush(stdout);
        drop(bi);
        drop(bo);
        meminfo("freed");
    }
    return 0;
}
