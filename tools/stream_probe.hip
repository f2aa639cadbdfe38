// stream_probe.hip — the zfec 4-of-8 memory pattern without the GF maths:
// per object, read 4 streams (shards at j*C) and write 8 streams (shards at
// j*SP, SP = C or C + pad), 16 B per lane per stream.  Sweeps workgroup size,
// tile schedule and store policy.  Calibration tool (not product code).
//   stream_probe [objects=1024] [K=4|8]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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
    uint64_t C, SP, in_stride, out_stride, count;
};

// MAP 0: grid-stride over tiles; 1: XCD-grouped; 3: XCD-grouped chunks of CH tiles
template <int TPB, int MAP, int CH, bool NT, bool SPLIT, int KS = 4>
__global__ __launch_bounds__(TPB) void k_stream(Args a) {
    constexpr uint64_t TILE = TPB * 16;
    const uint64_t tpo = a.C / TILE, T = tpo * a.count;
    const uint64_t G = gridDim.x, b = blockIdx.x;
    const uint64_t xb = (b % 8) * (G / 8) + b / 8;
    uint64_t c = (MAP == 0) ? b : xb;
    uint64_t tin = 0;
    for (;;) {
        uint64_t t;
        if (MAP == 3) {
            if (tin == CH) { c += G; tin = 0; }
            t = c * CH + tin++;
        } else {
            t = c;
            c += G;
        }
        if (t >= T) break;
        const uint64_t obj = t / tpo;
        const uint64_t col = (t - obj * tpo) * TILE + threadIdx.x * 16;
        const uint8_t *ib = a.in + obj * a.in_stride;
        uint8_t *ob = a.out + obj * a.out_stride;
        u32x4 v[KS];
#pragma unroll
        for (int j = 0; j < KS; ++j) v[j] = *(const u32x4 *)(ib + j * a.C + col);
#pragma unroll
        for (int j = 0; j < 2 * KS; ++j) {
            u32x4 w = j < KS ? v[j] : (v[j - KS] ^ 0x01020304u);
            uint8_t *p = ob + j * a.SP + col;
            if (SPLIT && j == KS) __builtin_amdgcn_s_waitcnt(0);
            if (NT) __builtin_nontemporal_store(w, (u32x4 *)p);
            else *(u32x4 *)p = w;
        }
    }
}

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 1024;
    const int KS = argc > 2 ? atoi(argv[2]) : 4;  // 4: 4-of-8 pattern, 8: 8-of-16
    const uint64_t C = (16ull << 20) / KS, n = KS * C;
    uint8_t *in, *out;
    const uint64_t PAD = 64 * 1024 + 4096;  // non-power-of-two shard spacing variant
    CK(hipMalloc(&in, count * n));
    CK(hipMalloc(&out, count * 2 * KS * (C + PAD)));
    CK(hipMemset(in, 7, count * n));
    CK(hipMemset(out, 0, count * 2 * KS * (C + PAD)));
    struct V {
        const char *name;
        void (*fn)(Args);
        int tpb, bpc;
        bool pad;
    };
#define VV(TPB, MAP, CH, NT, SPLIT, bpc, pad) \
    V{#TPB " MAP" #MAP " CH" #CH " NT" #NT " SPLIT" #SPLIT " bpc" #bpc " pad" #pad, k_stream<TPB, MAP, CH, NT, SPLIT>, TPB, bpc, pad}
#define V8(TPB, MAP, CH, NT, bpc) \
    V{"K8 " #TPB " MAP" #MAP " CH" #CH " NT" #NT " bpc" #bpc, k_stream<TPB, MAP, CH, NT, false, 8>, TPB, bpc, false}
    std::vector<V> vs8 = {
        V8(256, 3, 64, true, 1), V8(256, 3, 64, true, 2), V8(256, 3, 64, true, 4), V8(256, 3, 64, false, 2),
        V8(256, 3, 16, true, 2), V8(256, 1, 1, true, 2),  V8(256, 3, 64, false, 4), V8(512, 3, 32, true, 1),
        V8(128, 3, 128, true, 4), V8(128, 3, 128, true, 8),
    };
    std::vector<V> vs4 = {
        VV(256, 0, 1, true, false, 4, false),  VV(256, 1, 1, true, false, 4, false),
        VV(256, 3, 64, true, false, 4, false), VV(256, 3, 64, false, false, 4, false),
        VV(256, 1, 1, true, false, 4, true),   VV(256, 3, 64, true, false, 4, true),
        VV(1024, 1, 1, true, false, 1, false), VV(1024, 3, 16, true, false, 1, false),
        VV(1024, 3, 16, false, false, 1, false), VV(1024, 1, 1, true, false, 1, true),
        VV(512, 1, 1, true, false, 2, false),  VV(256, 1, 1, true, true, 4, false),
        VV(256, 1, 1, true, false, 2, false),  VV(256, 1, 1, true, false, 8, false),
    };
    std::vector<V> &vs = KS == 8 ? vs8 : vs4;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(vs.size());
    for (int rd = 0; rd < 5; ++rd)
        for (size_t i = 0; i < vs.size(); ++i) {
            Args a{in, out, C, vs[i].pad ? C + PAD : C, n, 2 * KS * (C + PAD), count};
            const int grid = 256 * vs[i].bpc;
            hipLaunchKernelGGL(vs[i].fn, dim3(grid), dim3(vs[i].tpb), 0, 0, a);
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(vs[i].fn, dim3(grid), dim3(vs[i].tpb), 0, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto t = ms[i];
        std::sort(t.begin(), t.end());
        printf("%-44s median %7.3f ms -> %7.1f GB/s\n", vs[i].name, t[2], 3.0 * count * n / (t[2] * 1e-3) / 1e9);
    }
    return 0;
}
