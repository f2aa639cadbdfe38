// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE on gfx950 for the read
// patterns of this repo (MI355X_MICROARCH.md: only 16-B-aligned streaming
// reads are calibrated, at 1/2).  Each kernel reads a known byte count once
// (4 GiB, beyond the 256 MiB Infinity Cache) and is dispatched once:
//   aligned16  : 16 B per lane, 16-B aligned, coalesced (the calibrated case)
//   shift8     : the same addresses + 8 B (bao stream slots sit at 8 mod 16:
//                K3 verify-decode's loads)
//   lines1k    : 8 lanes per 128-B line, one line per 1 KiB, 8 passes
//                (K13/K3's per-step chunk lines), 16-B aligned
// Run under: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a8 __attribute__((ext_vector_type(4), aligned(8)));

__global__ __launch_bounds__(256) void aligned16(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; i < bytes; i += (uint64_t)gridDim.x * 256 * 16) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void shift8(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; i + 16 < bytes; i += (uint64_t)gridDim.x * 256 * 16) {
        const u32x4_a8 v = *reinterpret_cast<const u32x4_a8 *>(p + 8 + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

// lane (g = lane / 8, l = lane % 8): bytes 128 s + 16 l of 1 KiB chunk (wave base + g)
__global__ __launch_bounds__(256) void lines1k(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64, lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    for (uint64_t c0 = wave * 8; (c0 + 8) * 1024 <= bytes; c0 += waves * 8)
        for (int s = 0; s < 8; ++s) {
            const u32x4 v = *reinterpret_cast<const u32x4 *>(p + (c0 + lane / 8) * 1024 + 128 * s + 16 * (lane % 8));
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t *p;
    uint32_t *sink;
    if (hipMalloc(&p, bytes + 256) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes + 256);
    hipLaunchKernelGGL(aligned16, dim3(2048), dim3(256), 0, 0, p, bytes, sink);
    hipLaunchKernelGGL(shift8, dim3(2048), dim3(256), 0, 0, p, bytes, sink);
    hipLaunchKernelGGL(lines1k, dim3(2048), dim3(256), 0, 0, p, bytes, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("each kernel read %llu bytes\n", (unsigned long long)bytes);
    return 0;
}
