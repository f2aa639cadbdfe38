// mix_probe.hip — the zfec 4-of-8 memory pattern (4 read + 8 write streams per
// object, 16 B per lane per stream, no GF maths) under store cache policies,
// wave counts, object-to-XCD placements and store orders that stream_probe /
// write_probe did not cover.  Calibration tool (not product code).
//   mix_probe [objects=1024] [rounds=5] [alloc: hip | bal]  (bal = the library's class-balanced allocator)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include <cstring>

#include "../carbonado_amd/csrc/hbm_alloc.hpp"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

struct Args {
    const uint8_t *in;
    uint8_t *out;
    uint64_t C, count;
};

// STORE: -1 flat nontemporal, 0 plain, >0 buffer-store aux bits (1 sc0, 2 nt, 16 sc1)
// LOADNT: input loads nontemporal.  MAP 3: XCD-grouped runs of CH tiles;
// MAP 4: object o is processed by the workgroups of XCD o % 8 only, which walk
// its tiles together (each XCD's write set = 8 sequential streams).
// ROT: wave w starts its 8 stores at shard (w % 8) (spread instantaneous streams).
template <int TPB, int MAP, int CH, int STORE, bool LOADNT, bool ROT, int NW = 8>
__global__ __launch_bounds__(TPB) void k_mix(Args a) {
    constexpr uint64_t TILE = TPB * 16;
    const uint64_t tpo = a.C / TILE, T = tpo * a.count;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const int wave = threadIdx.x / 64;
    uint64_t c, tin = 0, stride = G;
    if (MAP == 4) {
        // per XCD: G/8 workgroups, objects x, x+8, x+16, ... walked tile by tile
        const uint64_t x = b % 8, wi = b / 8, per = G / 8;
        c = wi;  // index within the XCD's tile list
        stride = per;
        (void)x;
    } else {
        c = (b % 8) * (G / 8) + b / 8;
    }
    const uint64_t xcd = b % 8;
    const uint64_t objs_x = (a.count + 7 - xcd) / 8;  // objects owned by this XCD (MAP 4)
    for (;;) {
        uint64_t t;
        if (MAP == 3) {
            if (tin == CH) { c += stride; tin = 0; }
            t = c * CH + tin++;
            if (t >= T) break;
        } else {
            t = c;
            c += stride;
            if (MAP == 4) {
                if (t >= objs_x * tpo) break;
                const uint64_t lo = t / tpo;
                t = (lo * 8 + xcd) * tpo + (t - lo * tpo);
            } else if (t >= T) break;
        }
        const uint64_t obj = t / tpo;
        const uint64_t col = (t - obj * tpo) * TILE + threadIdx.x * 16;
        const uint8_t *ib = a.in + obj * 4 * a.C;
        uint8_t *ob = a.out + obj * 8 * a.C;
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 *p = (const u32x4 *)(ib + j * a.C + col);
            v[j] = LOADNT ? __builtin_nontemporal_load(p) : *p;
        }
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(ob, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int jj = 0; jj < NW; ++jj) {
            const int j = ROT ? ((jj + wave) & 7) : jj;
            u32x4 w;
            if (ROT) {
                const u32x4 x0 = (j & 3) == 0 ? v[0] : (j & 3) == 1 ? v[1] : (j & 3) == 2 ? v[2] : v[3];
                w = j < 4 ? x0 : (x0 ^ 0x01020304u);
            } else {
                w = jj < 4 ? v[jj] : (v[jj - 4] ^ 0x01020304u);
            }
            const uint64_t off = (uint64_t)j * a.C + col;
            if (STORE < 0) __builtin_nontemporal_store(w, (u32x4 *)(ob + off));
            else if (STORE == 0) *(u32x4 *)(ob + off) = w;
            else __builtin_amdgcn_raw_buffer_store_b128(w, rb, (int)off, 0, STORE);
        }
    }
}

// the zfec 8-of-16 pattern: 8 read + 16 write streams per object (object =
// 8 shards of C2 bytes in, 16 out), XCD-grouped runs of CH tiles, nt stores
template <int TPB, int CH>
__global__ __launch_bounds__(TPB) void k_mix816(Args a) {
    constexpr uint64_t TILE = TPB * 16;
    const uint64_t C2 = a.C / 2, tpo = C2 / TILE, T = tpo * a.count, G = gridDim.x, b = blockIdx.x;
    uint64_t c = (b % 8) * (G / 8) + b / 8, tin = 0;
    for (;;) {
        if (tin == CH) { c += G; tin = 0; }
        const uint64_t t = c * CH + tin++;
        if (t >= T) break;
        const uint64_t obj = t / tpo, col = (t - obj * tpo) * TILE + threadIdx.x * 16;
        const uint8_t *ib = a.in + obj * 4 * a.C;
        uint8_t *ob = a.out + obj * 8 * a.C;
        u32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const u32x4 *)(ib + j * C2 + col);
#pragma unroll
        for (int j = 0; j < 16; ++j)
            __builtin_nontemporal_store(j < 8 ? v[j] : (v[j - 8] ^ 0x01020304u), (u32x4 *)(ob + j * C2 + col));
    }
}

// copy (1:1) and pure read / pure write references on the same buffers
__global__ __launch_bounds__(256) void k_read(const u32x4 *in, size_t n, u32x4 *sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= in[i];
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(in[i], out + i);
}
__global__ __launch_bounds__(256) void k_write(u32x4 *out, size_t n) {
    const u32x4 v = {1, 2, 3, (uint32_t)blockIdx.x};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) out[i] = v;
}

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t n = 16ull << 20, C = n / 4;
    uint8_t *in, *out;
    const bool bal = argc > 3 && !strcmp(argv[3], "bal");
    if (bal) {
        CK(chip::hbm::Allocator::get().alloc(count * n, reinterpret_cast<void **>(&in)));
        CK(chip::hbm::Allocator::get().alloc(count * 2 * n, reinterpret_cast<void **>(&out)));
    } else {
        CK(hipMalloc(&in, count * n));
        CK(hipMalloc(&out, count * 2 * n));
    }
    printf("buffers: %s\n", bal ? "class-balanced (hbm_alloc.hpp)" : "hipMalloc");
    CK(hipMemset(in, 7, count * n));
    CK(hipMemset(out, 0, count * 2 * n));
    struct V {
        std::string name;
        void (*fn)(Args);
        int tpb, grid;
        double bpi;  // bytes moved per input byte
    };
#define VV(TPB, MAP, CH, ST, LNT, ROT, BPC) \
    V{#TPB " MAP" #MAP " CH" #CH " st" #ST " lnt" #LNT " rot" #ROT " bpc" #BPC, k_mix<TPB, MAP, CH, ST, LNT, ROT>, TPB, 256 * BPC, 3.0}
#define V4(TPB, MAP, CH, ST, BPC) \
    V{"4r4w " #TPB " MAP" #MAP " CH" #CH " st" #ST " bpc" #BPC, k_mix<TPB, MAP, CH, ST, false, false, 4>, TPB, 256 * BPC, 2.0}
    std::vector<V> vs = {
        VV(256, 3, 64, -1, false, false, 4), VV(512, 3, 32, -1, false, false, 2),
        V4(256, 3, 64, -1, 4),               V4(256, 3, 64, 0, 4),
        V4(512, 3, 32, -1, 2),               V4(256, 3, 16, -1, 8),
        V{"8r16w 256 MAP3 CH32 st-1 bpc2", k_mix816<256, 32>, 256, 512, 3.0},
        V{"8r16w 256 MAP3 CH32 st-1 bpc4", k_mix816<256, 32>, 256, 1024, 3.0},
        V{"8r16w 512 MAP3 CH16 st-1 bpc2", k_mix816<512, 16>, 512, 512, 3.0},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto launch) {
        launch();
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        return t;
    };
    std::vector<std::vector<float>> ms(vs.size() + 3);
    for (int rd = 0; rd < rounds; ++rd) {
        for (size_t i = 0; i < vs.size(); ++i) {
            Args a{in, out, C, count};
            ms[i].push_back(timed([&] { hipLaunchKernelGGL(vs[i].fn, dim3(vs[i].grid), dim3(vs[i].tpb), 0, 0, a); }));
        }
        ms[vs.size()].push_back(timed([&] {
            hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, (const u32x4 *)in, count * n / 16, (u32x4 *)out);
        }));
        ms[vs.size() + 1].push_back(
            timed([&] { hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, (u32x4 *)out, count * 2 * n / 16); }));
        ms[vs.size() + 2].push_back(timed([&] {
            hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const u32x4 *)in, (u32x4 *)out, count * n / 16);
        }));
    }
    for (size_t i = 0; i < ms.size(); ++i) {
        auto t = ms[i];
        std::sort(t.begin(), t.end());
        const size_t x = i - vs.size();
        const char *name = i < vs.size() ? vs[i].name.c_str()
                           : x == 0      ? "read-only (input)"
                           : x == 1      ? "write-only (output)"
                                         : "copy 1:1 (input -> output, nt stores)";
        const double bytes = i < vs.size() ? vs[i].bpi * count * n : x == 0 ? 1.0 * count * n : 2.0 * count * n;
        printf("%-40s median %7.3f ms min %7.3f -> %7.1f GB/s (median) %7.1f (best)\n", name, t[t.size() / 2], t[0],
               bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / (t[0] * 1e-3) / 1e9);
    }
    return 0;
}
