// hbm_partition.hip — map which 1 GiB blocks of device memory write "together"
// fast.  hbm_regions showed writes confined to one 32 GiB half of a 64 GiB
// allocation at 5.4 TB/s and spread over both halves at 7.1 TB/s.  Here
// XCDs 0-3 write block r and XCDs 4-7 block j (nontemporal 16-B stores,
// 256 KiB runs): a pair much faster than (r, r) sits in different memory
// "partitions".  Calibration tool, not product.
//   hbm_partition [alloc_gib=32] [n_allocs=5] [block_mib=1024]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));          \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint64_t RUN = 256 << 10;

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }

// XCDs 0-3 write block a, XCDs 4-7 block b; each XCD a quarter of its block.
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

int main(int argc, char **argv) {
    const uint64_t alloc_gib = argc > 1 ? atoll(argv[1]) : 32;
    const int nalloc = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t block = (argc > 3 ? atoll(argv[3]) : 1024) << 20;
    std::vector<uint8_t *> allocs(nalloc);
    std::vector<uint8_t *> blocks;
    for (int i = 0; i < nalloc; ++i) {
        CK(hipMalloc(&allocs[i], alloc_gib << 30));
        CK(hipMemset(allocs[i], 0, alloc_gib << 30));
        for (uint64_t o = 0; o + block <= (alloc_gib << 30); o += block) blocks.push_back(allocs[i] + o);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_pair = [&](uint8_t *a, uint8_t *b) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(pair_write, dim3(512), dim3(256), 0, 0, a, b, block);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            best = std::min(best, t);
        }
        return (double)(2 * block) / (best * 1e-3) / 1e9;  // GB/s
    };
    const size_t nb = blocks.size();
    // pass 1: every block against block 0
    std::vector<double> r0(nb);
    for (size_t j = 0; j < nb; ++j) r0[j] = time_pair(blocks[0], blocks[j]);
    // class: "F" = fast with block 0 (other partition), "s" = slow (same)
    const double self = r0[0];
    size_t other = nb;
    printf("blocks of %llu MiB, %d allocations of %llu GiB; (0,0) = %.0f GB/s\n", (unsigned long long)(block >> 20),
           nalloc, (unsigned long long)alloc_gib, self);
    printf("pass 1, rate with block 0 (GB/s):\n");
    for (size_t j = 0; j < nb; ++j) {
        printf("%5.0f%s", r0[j], (j + 1) % 16 ? " " : "\n");
        if (other == nb && r0[j] > 1.1 * self) other = j;
    }
    printf("\n");
    if (other < nb) {
        printf("pass 2, rate with block %zu (GB/s):\n", other);
        for (size_t j = 0; j < nb; ++j) printf("%5.0f%s", time_pair(blocks[other], blocks[j]), (j + 1) % 16 ? " " : "\n");
        printf("\n");
    }
    // device pointers, for the physical-address guess
    for (int i = 0; i < nalloc; ++i) printf("alloc %d at %p\n", i, (void *)allocs[i]);
    return 0;
}
