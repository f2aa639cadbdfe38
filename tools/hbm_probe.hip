// hbm_probe.hip — measures achievable HBM bandwidth on this MI355X for the
// traffic mixes of the hot path (not product code; a calibration tool).
//   copy   : read 1 B, write 1 B
//   r1w2   : read 1 B, write 2 B (zfec 4-of-8 encode's mix: 16 MiB in, 32 MiB out)
//   r1w2nt : same with nontemporal stores
//   read   : read-only (xor reduce)
//   write  : write-only
// Usage: hbm_probe [GiB]   (default 4 GiB input, well beyond the 256 MiB MALL)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n) {
    size_t stride = (size_t)gridDim.x * 256 * UNROLL;
    for (size_t base = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x; base < n; base += stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = base + u * 256 < n ? in[base + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            if (base + u * 256 < n) {
                if (NT) __builtin_nontemporal_store(v[u], out + base + u * 256);
                else out[base + u * 256] = v[u];
            }
    }
}

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_r1w2(const u32x4 *__restrict__ in, u32x4 *__restrict__ a,
                                              u32x4 *__restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * 256 * UNROLL;
    for (size_t base = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x; base < n; base += stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = base + u * 256 < n ? in[base + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            if (base + u * 256 < n) {
                u32x4 w = v[u] ^ 0x5a5a5a5au;
                if (NT) {
                    __builtin_nontemporal_store(v[u], a + base + u * 256);
                    __builtin_nontemporal_store(w, b + base + u * 256);
                } else {
                    a[base + u * 256] = v[u];
                    b[base + u * 256] = w;
                }
            }
    }
}

__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ in, uint32_t *sink, size_t n) {
    size_t stride = (size_t)gridDim.x * 256 * 4;
    uint32_t acc = 0;
    for (size_t base = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; base < n; base += stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = base + u * 256 < n ? in[base + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(u32x4 *__restrict__ out, size_t n) {
    size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(u32x4{(uint32_t)i, 1, 2, 3}, out + i);
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    double gib = argc > 1 ? atof(argv[1]) : 4.0;
    size_t bytes = (size_t)(gib * (1ull << 30));
    size_t n = bytes / 16;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    u32x4 *in, *a, *b;
    uint32_t *sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    const int reps = 10;
    for (int blocks_per_cu : {4, 8, 16}) {
        int grid = cus * blocks_per_cu;
        float t;
        t = time_it([&] { hipLaunchKernelGGL((k_copy<4, false>), dim3(grid), dim3(256), 0, 0, in, a, n); }, reps);
        printf("grid=%5d copy      %8.1f GB/s (read+write)\n", grid, 2.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL((k_copy<4, true>), dim3(grid), dim3(256), 0, 0, in, a, n); }, reps);
        printf("grid=%5d copy_nt   %8.1f GB/s\n", grid, 2.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL((k_r1w2<4, false>), dim3(grid), dim3(256), 0, 0, in, a, b, n); }, reps);
        printf("grid=%5d r1w2      %8.1f GB/s\n", grid, 3.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL((k_r1w2<4, true>), dim3(grid), dim3(256), 0, 0, in, a, b, n); }, reps);
        printf("grid=%5d r1w2_nt   %8.1f GB/s\n", grid, 3.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL((k_r1w2<2, true>), dim3(grid), dim3(256), 0, 0, in, a, b, n); }, reps);
        printf("grid=%5d r1w2_nt_u2 %7.1f GB/s\n", grid, 3.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, in, sink, n); }, reps);
        printf("grid=%5d read      %8.1f GB/s\n", grid, 1.0 * bytes / t / 1e6);
        t = time_it([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, a, n); }, reps);
        printf("grid=%5d write_nt  %8.1f GB/s\n", grid, 1.0 * bytes / t / 1e6);
    }
    return 0;
}
