// bao_tune.hip — sweep K3/K4 variants (chunks per lane, stream-store policy)
// on a batch of 32 MiB objects, interleaved in one process.  Calibration tool.
//   bao_tune [objects=256] [mib=32] [rounds=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "bao_variants.hpp"

using namespace chip;
using namespace chip::bao;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

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

typedef hipError_t (*RunFn)(const uint8_t *, uint64_t, uint64_t, uint64_t, uint8_t *, uint64_t, uint8_t *,
                            uint32_t *, void *, hipStream_t, size_t, uint64_t);

struct V {
    std::string name;
    RunFn fn;
    int cpl;
    bool stream;
    size_t pad_lds;
};

template <int MODE, int CPL, bool NTS, int SP = 0, int SU = 1, int SE = 0, int XG = 0, bool DQ = false>
V mk(bool stream, size_t pad_lds = 0) {
    char b[96];
    snprintf(b, sizeof b, "%s CPL%d %s %s sp%d su%d se%d xg%d dq%d pad%zu", MODE == 3 ? "in-place" : MODE ? "decode" : "encode",
             CPL, NTS ? "nt " : "pln", stream ? "stream" : "hash-only", SP, SU, SE, XG, (int)DQ, pad_lds);
    return V{b, run_bao_t<MODE, CPL, NTS, SP, SU, SE, XG, DQ>, CPL, stream, pad_lds};
}

namespace chip {
int num_cus() { return 256; }
// run-queue counters for the DQ (persistent) variants: one zeroed block, as the library's per-stream one
hipError_t stream_queue(hipStream_t, uint32_t **out) {
    static uint32_t *q = nullptr;
    if (!q) {
        hipError_t e = hipMalloc(&q, 4096);
        if (e != hipSuccess) return e;
        if ((e = hipMemset(q, 0, 4096)) != hipSuccess) return e;
    }
    *out = q;
    return hipSuccess;
}
}  // namespace chip

int main(int argc, char **argv) {
    const uint64_t count = argc > 1 ? atoll(argv[1]) : 256;
    const uint64_t n = (argc > 2 ? atoll(argv[2]) : 32) << 20;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const uint64_t blen = 8 + n + 64 * (n_chunks(n) - 1);
    const uint64_t oal = argc > 5 ? atoll(argv[5]) : 256;  // output stride alignment (bytes)
    const uint64_t ostride = (blen + oal - 1) / oal * oal;
    uint8_t *in, *out, *hash, *dec, *scratch;
    uint32_t *status;
    CK(hipMalloc(&in, count * n));
    CK(hipMalloc(&out, count * ostride));
    CK(hipMalloc(&dec, count * n));
    CK(hipMalloc(&hash, count * 32));
    CK(hipMalloc(&status, count * 4));
    CK(hipMalloc(&scratch, bao_scratch_len_t<1>(n, count)));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t *)in, count * n / 8, 0xB1A3ull);
    // product encode / decode / in-place, each with the XCD-grouped block order (XG 1)
    // encode with the stream (SP 3, the non-64-KiB-multiple path), decode (product: CPL 2, nt content
    // stores, XG 1, DQ), hash-only encode for the VALU ceiling.  A decode variant issuing the content
    // stores after the next step's loads (read back from the rows) measured the same (r2x_bao_tune.txt)
    std::vector<V> vs = {mk<0, 2, false, 3, 8, 0, 1, true>(true), mk<1, 2, true, 0, 1, 0, 1, true>(true),
                         mk<0, 2, false, 0, 1, 0, 1, true>(false),
                         // round 4: decode without the duplicated border-line fetches
                         // (diagnostic, wrong output), then the product again
                         mk<1, 2, true, 0, 1, 6, 1, true>(true), mk<1, 2, true, 0, 1, 0, 1, true>(true)};
    // earlier: product encode / decode / in-place with XG 0 and 1 (profiles/r1x_ab_bao_xcd_order.txt)
    // round-1 store diagnostics (profiles/r1x_bao_store_diagnostics.txt): mk<0, 2, false>(false) hash-only,
    // mk<0, 2, false, 3, 1, SE>(true) for SE 2..5, mk<0, 1, false, 3>(true), mk<1, 1, false>(true)
    if (argc > 4) {  // comma-separated subset of variant indices (profiling)
        std::vector<V> keep;
        std::string sel = argv[4];
        size_t pos = 0;
        while (pos <= sel.size()) {
            size_t e = sel.find(',', pos);
            if (e == std::string::npos) e = sel.size();
            keep.push_back(vs[atoi(sel.substr(pos, e - pos).c_str())]);
            pos = e + 1;
        }
        vs = keep;
    }
    unsigned long long *dsum;
    CK(hipMalloc(&dsum, 8));
    std::vector<std::vector<float>> ms(vs.size());
    unsigned long long ref_stream = 0, ref_hash = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // reference encode (CPL1) so decode variants have a stream + hashes to verify
    CK((run_bao_t<0, 1, false>(in, n, n, count, out, ostride, hash, nullptr, scratch, 0, 0)));
    CK(hipDeviceSynchronize());
    for (int rd = 0; rd < rounds; ++rd)
        for (size_t v = 0; v < vs.size(); ++v) {
            const bool dec_mode = vs[v].name[0] == 'd';
            const bool inplace = vs[v].name[0] == 'i';
            auto launch = [&] {
                if (inplace) {
                    CK(vs[v].fn(out, ostride, n, count, out, ostride, hash, nullptr, scratch, 0, vs[v].pad_lds, ~0ull));
                } else if (dec_mode) {
                    CK(hipMemsetAsync(status, 0, count * 4, 0));
                    CK(vs[v].fn(out, ostride, n, count, dec, n, hash, status, scratch, 0, vs[v].pad_lds, ~0ull));
                } else {
                    CK(vs[v].fn(in, n, n, count, vs[v].stream ? out : nullptr, ostride, hash, nullptr, scratch, 0,
                                vs[v].pad_lds, ~0ull));
                }
            };
            launch();
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t);
            if (rd == 0) {
                unsigned long long hs, ss = 0;
                CK(hipMemset(dsum, 0, 8));
                hipLaunchKernelGGL(checksum_kernel, dim3(64), dim3(256), 0, 0, (const uint64_t *)hash, count * 4, dsum);
                CK(hipMemcpy(&hs, dsum, 8, hipMemcpyDeviceToHost));
                if (vs[v].stream && !dec_mode && !inplace) {
                    CK(hipMemset(dsum, 0, 8));
                    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)out,
                                       count * ostride / 8, dsum);
                    CK(hipMemcpy(&ss, dsum, 8, hipMemcpyDeviceToHost));
                }
                if (v == 0) { ref_hash = hs; ref_stream = ss; }
                if (hs != ref_hash) printf("!! %s hash mismatch\n", vs[v].name.c_str());
                if (vs[v].stream && !dec_mode && !inplace && ss != ref_stream) printf("!! %s stream mismatch\n", vs[v].name.c_str());
                if (dec_mode) {
                    std::vector<uint32_t> st(count);
                    CK(hipMemcpy(st.data(), status, count * 4, hipMemcpyDeviceToHost));
                    for (auto x : st)
                        if (x) { printf("!! %s status %u\n", vs[v].name.c_str(), x); break; }
                    unsigned long long a = 0, b = 0;
                    CK(hipMemset(dsum, 0, 8));
                    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)dec, count * n / 8, dsum);
                    CK(hipMemcpy(&a, dsum, 8, hipMemcpyDeviceToHost));
                    CK(hipMemset(dsum, 0, 8));
                    hipLaunchKernelGGL(checksum_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t *)in, count * n / 8, dsum);
                    CK(hipMemcpy(&b, dsum, 8, hipMemcpyDeviceToHost));
                    if (a != b) printf("!! %s decoded content mismatch\n", vs[v].name.c_str());
                }
            }
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto t = ms[v];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2];
        printf("%-34s median %8.3f ms -> %7.1f GB/s hashed, %7.1f GiB/s\n", vs[v].name.c_str(), med,
               (double)count * n / (med * 1e-3) / 1e9, (double)count * n / (med * 1e-3) / (1 << 30));
    }
    return 0;
}
