// write_probe.hip — which store pattern / cache policy writes HBM fastest on
// this MI355X?  Calibration tool for K1 (not product code).
//   write_probe [GiB=8]
// Each workgroup (256 threads, 16 B per lane per store) writes contiguous
// chunks of CHUNK bytes; chunks are dealt to workgroups grid-stride, or
// XCD-grouped (the G/8 blocks with equal b%8 take consecutive chunks).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// AUX: buffer-store cache-policy bits (gfx950): 1 = sc0, 2 = nt, 16 = sc1; -1 = flat nontemporal builtin
template <int AUX, bool XCD, bool READ>
__global__ __launch_bounds__(256) void k_write(uint8_t *out, const uint8_t *in, size_t bytes, size_t chunk) {
    const size_t nchunks = bytes / chunk;
    const size_t G = gridDim.x, b = blockIdx.x;
    size_t it = 0;
    const size_t per = G / 8;
    for (;; ++it) {
        size_t c = XCD ? it * G + (b % 8) * per + b / 8 : it * G + b;
        if (c >= nchunks) break;
        uint8_t *base = out + c * chunk;
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
        for (size_t off = threadIdx.x * 16; off < chunk; off += 256 * 16 * 4) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (READ) v[u] = off + u * 4096 < chunk ? *(const u32x4 *)(in + c * chunk + off + u * 4096) : u32x4{0, 0, 0, 0};
                else v[u] = u32x4{(uint32_t)(c + off), (uint32_t)u, 7u, 9u};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint8_t *p = base + off + u * 4096;
                if (off + u * 4096 >= chunk) break;
                if (AUX < 0) __builtin_nontemporal_store(v[u], (u32x4 *)p);
                else if (AUX == 0) *(u32x4 *)p = v[u];
                else __builtin_amdgcn_raw_buffer_store_b128(v[u], rb, (int)(off + u * 4096), 0, AUX);
            }
        }
    }
}

template <typename F>
float time_it(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    return best;
}

int main(int argc, char **argv) {
    double gib = argc > 1 ? atof(argv[1]) : 8.0;
    size_t bytes = (size_t)(gib * (1ull << 30));
    uint8_t *out, *in;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&in, bytes));
    CK(hipMemset(out, 0, bytes));
    CK(hipMemset(in, 3, bytes));
#define RUN(AUX, XCD, READ, label)                                                                      \
    for (size_t chunk : {4096ul, 16384ul, 65536ul, 262144ul, 1048576ul})                               \
        for (int bpc : {2, 4, 8}) {                                                                     \
            int grid = 256 * bpc;                                                                       \
            float t = time_it([&] {                                                                     \
                hipLaunchKernelGGL((k_write<AUX, XCD, READ>), dim3(grid), dim3(256), 0, 0, out, in,     \
                                   bytes, chunk);                                                       \
            });                                                                                         \
            printf("%-14s chunk %7zu bpc %d : %7.1f GB/s\n", label, chunk, bpc,                         \
                   (READ ? 2.0 : 1.0) * bytes / (t * 1e-3) / 1e9);                                      \
        }
    RUN(-1, false, false, "nt-flat");
    RUN(-1, true, false, "nt-flat-xcd");
    RUN(0, true, false, "plain-xcd");
    RUN(2, true, false, "buf-nt-xcd");
    RUN(16, true, false, "buf-sc1-xcd");
    RUN(17, true, false, "buf-sc0sc1-xcd");
    RUN(18, true, false, "buf-ntsc1-xcd");
    RUN(3, true, false, "buf-ntsc0-xcd");
    RUN(-1, true, true, "copy-nt-xcd");
    return 0;
}
