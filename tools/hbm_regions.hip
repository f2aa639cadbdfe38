// hbm_regions.hip — does the HBM rate depend on WHERE in a large allocation
// the concurrent traffic lands?  Each XCD streams its own 4 GiB region
// (reads or nontemporal 16-B writes, 256 KiB runs per workgroup, 2
// workgroups/CU), region bases chosen per configuration inside one 64 GiB
// buffer; all configurations interleaved in one process.  Calibration tool,
// not product.
//   hbm_regions [rounds=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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
constexpr uint64_t GiB = 1ull << 30;
constexpr uint64_t RUN = 256 << 10;  // bytes per workgroup run

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }

struct Args {
    uint8_t *buf;
    uint64_t base[8];  // byte offset of each XCD's region
    uint64_t bytes;    // per XCD
    uint64_t *trace;   // per XCD: max end (wall clock)
    uint32_t *sink;
};

// Workgroup w of XCD x walks runs w, w + g, ... of its XCD's region (g = workgroups on the XCD).
template <bool WRITE>
__global__ __launch_bounds__(256) void stream_kernel(Args a) {
    const uint32_t x = xcc_id();
    const uint32_t g = gridDim.x / 8, w = blockIdx.x / 8;
    uint8_t *reg = a.buf + a.base[x];
    const uint64_t runs = a.bytes / RUN;
    u32x4 acc = {0u, 0u, 0u, 0u};
    const u32x4 val = {blockIdx.x, threadIdx.x, 1u, 2u};
    for (uint64_t r = w; r < runs; r += g) {
        uint8_t *p = reg + r * RUN + threadIdx.x * 16;
#pragma unroll 4
        for (int i = 0; i < (int)(RUN / 4096); ++i) {
            if (WRITE) __builtin_nontemporal_store(val, reinterpret_cast<u32x4 *>(p + i * 4096));
            else acc ^= *reinterpret_cast<const u32x4 *>(p + i * 4096);
        }
    }
    if (!WRITE && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) a.sink[0] = 1;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned long long *>(a.trace + x), wall_clock64());
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    uint8_t *buf;
    CK(hipMalloc(&buf, 64 * GiB));
    CK(hipMemset(buf, 1, 64 * GiB));
    uint64_t *trace;
    uint32_t *sink;
    CK(hipMalloc(&trace, 64));
    CK(hipMalloc(&sink, 64));
    struct Cfg { std::string name; uint64_t base_gib[8]; };
    std::vector<Cfg> cfgs = {
        {"all in [0,32): x*4", {0, 4, 8, 12, 16, 20, 24, 28}},
        {"all in [32,64): 32+x*4", {32, 36, 40, 44, 48, 52, 56, 60}},
        {"split: x*8", {0, 8, 16, 24, 32, 40, 48, 56}},
        {"x<4 low, x>=4 high", {0, 4, 8, 12, 32, 36, 40, 44}},
        {"even low, odd high", {0, 32, 4, 36, 8, 40, 12, 44}},
        {"[16,48): 16+x*4", {16, 20, 24, 28, 32, 36, 40, 44}},
        {"all in [0,16) x*2", {0, 2, 4, 6, 8, 10, 12, 14}},
        {"all in [16,32) 16+x*2", {16, 18, 20, 22, 24, 26, 28, 30}},
        {"all in [32,48) 32+x*2", {32, 34, 36, 38, 40, 42, 44, 46}},
        {"all in [48,64) 48+x*2", {48, 50, 52, 54, 56, 58, 60, 62}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int wr = 0; wr < 2; ++wr) {
        std::vector<std::vector<float>> ms(cfgs.size());
        std::vector<std::vector<double>> xend(cfgs.size(), std::vector<double>(8, 0));
        for (int rd = 0; rd < rounds; ++rd)
            for (size_t c = 0; c < cfgs.size(); ++c) {
                Args a{};
                a.buf = buf;
                // [0,16)-style configurations stream 2 GiB per XCD, the others 4 GiB
                a.bytes = (cfgs[c].base_gib[1] - cfgs[c].base_gib[0] == 2) ? 2 * GiB : 4 * GiB;
                for (int x = 0; x < 8; ++x) a.base[x] = cfgs[c].base_gib[x] * GiB;
                a.trace = trace;
                a.sink = sink;
                auto fn = wr ? stream_kernel<true> : stream_kernel<false>;
                CK(hipMemset(trace, 0, 64));
                uint64_t t0 = 0;
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(fn, dim3(512), dim3(256), 0, 0, a);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[c].push_back(t * 4.0f * GiB / a.bytes);  // normalised to 4 GiB per XCD
                uint64_t h[8];
                CK(hipMemcpy(h, trace, 64, hipMemcpyDeviceToHost));
                t0 = *std::min_element(h, h + 8);
                for (int x = 0; x < 8; ++x) xend[c][x] = (h[x] - t0) * 1e-5;
            }
        printf("== %s, 8 XCDs x 4 GiB (times normalised to 32 GiB)\n", wr ? "WRITE nt" : "READ");
        for (size_t c = 0; c < cfgs.size(); ++c) {
            auto t = ms[c];
            std::sort(t.begin(), t.end());
            printf("%-26s median %7.3f ms -> %7.1f GB/s | XCD end spread ms:", cfgs[c].name.c_str(), t[t.size() / 2],
                   32.0 * GiB / (t[t.size() / 2] * 1e-3) / 1e9);
            for (int x = 0; x < 8; ++x) printf(" %.2f", xend[c][x]);
            printf("\n");
        }
    }
    return 0;
}
