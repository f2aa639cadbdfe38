// bar_probe.hip — can the host write a single object's bytes straight into
// device memory over PCIe (fine-grained / uncached VRAM mapped through the
// BAR), and at what rate, against the KM path's two steps (host copy into
// pinned host memory, then the kernel reading it over PCIe at ~26 GB/s)?
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/bar_probe.hip -o tools/bar_probe -lpthread
//   bar_probe [BYTES] [REPS]
// Prints per allocation kind: whether the host can address it, host write
// rate with 1 and 8 threads (AVX2 streaming stores), the device's read rate
// of the same bytes, and a checksum cross-check of what the device read.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::printf("  %s -> %s\n", #x, hipGetErrorString(e_));                               \
            return false;                                                                         \
        }                                                                                         \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__attribute__((target("avx2"))) static void nt_copy(uint8_t *d, const uint8_t *s, size_t n) {
    size_t i = 0;
    for (; i + 32 <= n; i += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i)));
    std::memcpy(d + i, s + i, n - i);
    _mm_sfence();
}

static void host_write(uint8_t *dst, const uint8_t *src, size_t n, int threads) {
    if (threads == 1) {
        nt_copy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([=] {
            const size_t a = (n * t / threads) & ~size_t(63), b = t + 1 == threads ? n : (n * (t + 1) / threads) & ~size_t(63);
            nt_copy(dst + a, src + a, b - a);
        });
    for (auto &x : th) x.join();
}

// every thread sums its 16-B words; one atomic per block into *out (vector atomics only)
__global__ void read_sum(const uint4 *p, size_t words, unsigned long long *out) {
    unsigned long long s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        s += (unsigned long long)v.x + v.y + v.z + v.w;
    }
    __shared__ unsigned long long part[256];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < (int)blockDim.x; ++i) t += part[i];
        atomicAdd(out, t);
    }
}

// KM's read pattern (multi_kernels.hip phase 2): a quad of lanes per 1 KiB
// chunk, lane q loading bytes 64 b + 16 q of every block b, all 16 loads in
// flight; 64 chunks per workgroup of 256 threads.
__global__ __launch_bounds__(256) void read_km(const uint4 *p, size_t chunks, unsigned long long *out) {
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const size_t c = blockIdx.x * (size_t)64 + g;
    unsigned long long s = 0;
    if (c < chunks) {
        uint4 v[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) v[b] = p[c * 64 + 4 * b + q];
#pragma unroll
        for (int b = 0; b < 16; ++b) s += (unsigned long long)v[b].x + v[b].y + v[b].z + v[b].w;
    }
    __shared__ unsigned long long part[256];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        unsigned long long u = 0;
        for (int i = 0; i < 256; ++i) u += part[i];
        atomicAdd(out, u);
    }
}

// the same 64 chunks per workgroup, but each wave instruction reads one whole
// chunk (lane L: bytes 16 L .. 16 L + 15): wave w loads chunks 16 w .. 16 w + 15
__global__ __launch_bounds__(256) void read_rows(const uint4 *p, size_t chunks, unsigned long long *out) {
    const int t = threadIdx.x, w = t >> 6, L = t & 63;
    unsigned long long s = 0;
    uint4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const size_t c = blockIdx.x * (size_t)64 + 16 * w + i;
        v[i] = c < chunks ? p[c * 64 + L] : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s += (unsigned long long)v[i].x + v[i].y + v[i].z + v[i].w;
    __shared__ unsigned long long part[256];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        unsigned long long u = 0;
        for (int i = 0; i < 256; ++i) u += part[i];
        atomicAdd(out, u);
    }
}

// one lane stores `v` to a pinned host word with system scope (vector store)
__global__ void flag_kernel(unsigned *flag, unsigned v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// host-side completion latency of a trivial launch: hipStreamSynchronize
// against spinning on a flag the kernel writes to pinned memory (then the
// synchronize, which returns at once)
static bool sync_latency(int reps) {
    std::printf("== completion latency of a one-lane kernel\n");
    unsigned *flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocDefault));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<double> ts, tf, tf2;
    for (int r = 0; r < reps; ++r) {
        __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
        double a = now_us();
        flag_kernel<<<1, 64, 0, s>>>(flag, 1u);
        CK(hipStreamSynchronize(s));
        ts.push_back(now_us() - a);
        __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
        a = now_us();
        flag_kernel<<<1, 64, 0, s>>>(flag, 2u);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != 2u) _mm_pause();
        tf.push_back(now_us() - a);
        CK(hipStreamSynchronize(s));
        tf2.push_back(now_us() - a);
    }
    std::sort(ts.begin(), ts.end());
    std::sort(tf.begin(), tf.end());
    std::sort(tf2.begin(), tf2.end());
    std::printf("  launch + hipStreamSynchronize: median %.1f us (p10 %.1f, p90 %.1f)\n", ts[ts.size() / 2],
                ts[ts.size() / 10], ts[ts.size() * 9 / 10]);
    std::printf("  launch + spin on the flag:     median %.1f us (p10 %.1f, p90 %.1f); + the synchronize %.1f us\n",
                tf[tf.size() / 2], tf[tf.size() / 10], tf[tf.size() * 9 / 10], tf2[tf2.size() / 2]);
    CK(hipStreamDestroy(s));
    CK(hipHostFree(flag));
    return true;
}

// pinned -> pinned and pinned -> HBM copies, 16 B per lane, all loads first
__global__ void copy16(const uint4 *src, uint4 *dst, size_t words) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < words) dst[i] = src[i];
}

template <class F>
static bool time_kernel(const char *what, size_t n, int reps, unsigned long long want, unsigned long long *dsum, F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> kt;
    unsigned long long got = 0;
    for (int r = 0; r < reps; ++r) {
        CK(hipMemset(dsum, 0, 8));
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        kt.push_back(ms * 1e3f);
        CK(hipMemcpy(&got, dsum, 8, hipMemcpyDeviceToHost));
    }
    std::sort(kt.begin(), kt.end());
    std::printf("  %-34s median %7.1f us = %5.1f GB/s, checksum %s\n", what, kt[kt.size() / 2],
                n / kt[kt.size() / 2] / 1e3, got == want ? "ok" : "MISMATCH");
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return true;
}

static bool patterns(size_t n, int reps, const std::vector<uint8_t> &src, unsigned long long want) {
    std::printf("== read patterns over pinned host memory (%zu B)\n", n);
    void *h = nullptr;
    CK(hipHostMalloc(&h, n, hipHostMallocDefault));
    std::memcpy(h, src.data(), n);
    void *dv = nullptr;
    CK(hipMalloc(&dv, n));
    CK(hipMemcpy(dv, src.data(), n, hipMemcpyHostToDevice));
    unsigned long long *dsum = nullptr;
    CK(hipMalloc(&dsum, 8));
    const size_t chunks = n / 1024;
    const unsigned G = (unsigned)((chunks + 63) / 64);
    const uint4 *hp = static_cast<const uint4 *>(h), *vp = static_cast<const uint4 *>(dv);
    time_kernel("KM quads (pinned)", n, reps, want, dsum, [&] { read_km<<<G, 256>>>(hp, chunks, dsum); });
    time_kernel("whole-chunk rows (pinned)", n, reps, want, dsum, [&] { read_rows<<<G, 256>>>(hp, chunks, dsum); });
    time_kernel("grid-stride 256 WG (pinned)", n, reps, want, dsum, [&] { read_sum<<<256, 256>>>(hp, n / 16, dsum); });
    time_kernel("grid-stride 32 WG (pinned)", n, reps, want, dsum, [&] { read_sum<<<32, 256>>>(hp, n / 16, dsum); });
    time_kernel("KM quads (HBM)", n, reps, want, dsum, [&] { read_km<<<G, 256>>>(vp, chunks, dsum); });
    {
        void *h2 = nullptr;
        CK(hipHostMalloc(&h2, n, hipHostMallocDefault));
        const unsigned cg = (unsigned)((n / 16 + 255) / 256);
        time_kernel("copy pinned -> pinned (read+write)", n, reps, want, dsum, [&] {
            copy16<<<cg, 256>>>(hp, static_cast<uint4 *>(h2), n / 16);
            read_sum<<<256, 256>>>(vp, n / 16, dsum);  // (the checksum from HBM: the timing is the copy's + ~6 us)
        });
        time_kernel("copy pinned -> HBM", n, reps, want, dsum, [&] {
            copy16<<<cg, 256>>>(hp, static_cast<uint4 *>(dv), n / 16);
            read_sum<<<256, 256>>>(vp, n / 16, dsum);
        });
        time_kernel("copy HBM -> pinned", n, reps, want, dsum, [&] {
            copy16<<<cg, 256>>>(vp, static_cast<uint4 *>(h2), n / 16);
            read_sum<<<256, 256>>>(vp, n / 16, dsum);
        });
        CK(hipHostFree(h2));
    }
    time_kernel("whole-chunk rows (HBM)", n, reps, want, dsum, [&] { read_rows<<<G, 256>>>(vp, chunks, dsum); });
    CK(hipFree(dsum));
    CK(hipFree(dv));
    CK(hipHostFree(h));
    return true;
}

static bool probe(const char *name, unsigned flags, bool host_alloc, size_t n, int reps, const std::vector<uint8_t> &src,
                  unsigned long long want) {
    std::printf("== %s\n", name);
    void *d = nullptr;
    if (host_alloc) CK(hipHostMalloc(&d, n, hipHostMallocDefault));
    else CK(hipExtMallocWithFlags(&d, n, flags));
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, d));
    void *hp = at.hostPointer;
    std::printf("  type %d device %p host %p\n", (int)at.type, at.devicePointer, hp);
    unsigned long long *dsum = nullptr;
    CK(hipMalloc(&dsum, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (!hp) {
        std::printf("  not host-addressable: skipped\n");
    } else {
        for (int threads : {1, 8}) {
            std::vector<double> t;
            for (int r = 0; r < reps; ++r) {
                const double a = now_us();
                host_write(static_cast<uint8_t *>(hp), src.data(), n, threads);
                t.push_back(now_us() - a);
            }
            std::sort(t.begin(), t.end());
            std::printf("  host write %zu B, %d thread(s): median %.1f us = %.1f GB/s\n", n, threads, t[t.size() / 2],
                        n / t[t.size() / 2] / 1e3);
        }
        std::vector<float> kt;
        unsigned long long got = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(dsum, 0, 8));
            CK(hipEventRecord(e0, 0));
            read_sum<<<256, 256>>>(static_cast<const uint4 *>(at.devicePointer ? at.devicePointer : d), n / 16, dsum);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            kt.push_back(ms * 1e3f);
            CK(hipMemcpy(&got, dsum, 8, hipMemcpyDeviceToHost));
        }
        std::sort(kt.begin(), kt.end());
        std::printf("  device read: median %.1f us = %.1f GB/s, checksum %s\n", kt[kt.size() / 2],
                    n / kt[kt.size() / 2] / 1e3, got == want ? "ok" : "MISMATCH");
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(dsum));
    if (host_alloc) CK(hipHostFree(d));
    else CK(hipFree(d));
    return true;
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) / 64 * 64 : (size_t(2) << 20);
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    std::vector<uint8_t> src(n);
    unsigned long long want = 0;
    for (size_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 131 + 7);
    for (size_t i = 0; i < n; i += 4) {
        uint32_t w;
        std::memcpy(&w, &src[i], 4);
        want += w;
    }
    sync_latency(200);
    patterns(n, reps, src, want);
    probe("pinned host memory (the KM path today)", 0, true, n, reps, src, want);
    probe("VRAM fine-grained", hipDeviceMallocFinegrained, false, n, reps, src, want);
    probe("VRAM uncached", hipDeviceMallocUncached, false, n, reps, src, want);
    probe("VRAM default (coarse-grained)", hipDeviceMallocDefault, false, n, reps, src, want);
    return 0;
}
