// reuse_probe.hip — do re-reads at a short reuse distance reach HBM?
//
// Verify-decode (K3 MODE 1) reads some 64-B segments of the stream twice:
// the segment a chunk step's last lane touches for 8 bytes is read again,
// whole, one step later (DESIGN §6 "Verify-decode traffic").  FETCH_SIZE
// counts the second read (the L2 has evicted the line by then), but the
// guide (MI355X_MICROARCH.md, Infinity Cache) says a line stays in the 256 MiB
// Infinity Cache while everything loaded or stored between its two uses
// fits in it.  This probe measures that rule on the box: a streaming read of
// a buffer, and the same read with every 16-B piece read a second time
// `lag` bytes later in the stream (all lanes advance through the buffer
// together, so the reuse distance is ~lag bytes of chip-wide traffic).
// If the second reads come from the Infinity Cache, the time stays at the
// single-read time while FETCH_SIZE doubles; once lag passes ~256 MiB they
// come from HBM and the time doubles too.
//
// Build: hipcc -O3 --offload-arch=gfx950 tools/reuse_probe.hip -o tools/reuse_probe
// Run:   tools/reuse_probe [GiB=8]   (time per variant; rocprofv3 --pmc FETCH_SIZE for the counters)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// lag == 0: one read of every piece; else piece i is read again at i + lag
// (the loop reads i and i - lag together)
__global__ __launch_bounds__(256) void reuse_kernel(const u32x4 *buf, uint64_t nvec, uint64_t lagvec, uint32_t *out) {
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += stride) {
        acc ^= buf[i];
        if (lagvec && i >= lagvec) acc ^= buf[i - lagvec];
    }
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x9E3779B9u) out[0] = r;  // keep the loads alive
}

__global__ void fill_kernel(uint64_t *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char **argv) {
    const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 8;
    const uint64_t bytes = gib << 30, nvec = bytes / 16;
    uint8_t *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 4));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)buf, bytes / 8);
    CK(hipDeviceSynchronize());
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const unsigned grid = (unsigned)p.multiProcessorCount * 8;
    const uint64_t lags_mib[] = {0, 1, 4, 16, 64, 128, 192, 256, 384, 512, 1024, 2048};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("buffer %llu GiB, grid %u x 256; reads: the buffer once, plus a second read of each piece lag MiB later\n",
           (unsigned long long)gib, grid);
    for (uint64_t lm : lags_mib) {
        const uint64_t lagvec = (lm << 20) / 16;
        if (lagvec >= nvec) continue;
        std::vector<float> t;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(reuse_kernel, dim3(grid), dim3(256), 0, 0, (const u32x4 *)buf, nvec, lagvec, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[2];
        const double reread = lagvec ? (double)(nvec - lagvec) * 16 : 0.0;  // bytes read twice
        printf("lag %5llu MiB  %8.3f ms  first reads %6.2f TB/s  all reads %6.2f TB/s  (re-read bytes %.2f GB)\n",
               (unsigned long long)lm, ms, bytes / (ms * 1e-3) / 1e12, (bytes + reread) / (ms * 1e-3) / 1e12,
               reread / 1e9);
        fflush(stdout);
    }
    return 0;
}
