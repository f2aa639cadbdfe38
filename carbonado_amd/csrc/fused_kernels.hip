// fused_kernels.hip — host side of K13 (fused_device.hpp): encode() at
// Zfec|Bao as one zfec+hash pass, then the parent levels (K4 / K4t).
#include "chip_internal.hpp"
#include "fused_device.hpp"

#include <algorithm>
#include <cstdlib>

namespace chip {

uint64_t zfec_bao_scratch_len(uint64_t zlen, uint64_t count) {
    const uint64_t N = bao::n_chunks(zlen);
    return count * 32 * (N + (N + 1) / 2);
}

namespace {

// K13 with 32-bit per-lane offsets from the object bases (O32) and the
// packed GF table addresses (GFP); -DK13_O32_DEF=0 / -DK13_GFP_DEF=0 build
// the 64-bit-address / per-byte-address forms for A/B.
#ifndef K13_O32_DEF
#define K13_O32_DEF 1
#endif
#ifndef K13_GFP_DEF
#define K13_GFP_DEF 1
#endif
#ifndef K13_NTL_DEF
#define K13_NTL_DEF 1
#endif
constexpr bool K13_O32 = K13_O32_DEF;
constexpr int K13_GFP = K13_GFP_DEF;
// content mode (bao of the content, KIND 1): input loads nontemporal, +1.5-1.9 %
// (A/B r7u); the zfec+bao kernels keep plain loads (FULL path even, general
// path -2..-4 % with them)
constexpr bool K13_NTL = K13_NTL_DEF;
// the stream of an object of shard length C is < 8.6 C bytes and its input
// 4 C: 32-bit offsets for C < 256 MiB.  CHIP_K13_O32=0 (read per call, so a
// test can flip it) takes the 64-bit-address kernels at any size.
bool o32_ok(uint64_t C_or_n) {
    const char *e = std::getenv("CHIP_K13_O32");
    if (e && e[0] == '0' && e[1] == 0) return false;
    return C_or_n < (1ull << 28);
}

}  // namespace

namespace fused {

// The product's K13 configurations (fused_device.hpp documents the template
// arguments): encode() at Zfec|Bao with levels 1-3 in the wave (FULL) or from
// the level-0 CVs (general: 8 does not divide the shard's chunk count, or
// zfec padding; both message words of a step read at once, MP 1: -1.5 %
// kernel time, tools/fused_tune, profiles/r6f/r6h/r6i; the FULL path measured
// no gain from it), and bao of the content (KIND 1).  _a64: 64-bit addresses
// for shards of 256 MiB and more.
__global__ __launch_bounds__(fused::FTPB) void zfec_bao_fused_kernel_full(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, true, 1, 0, 0, true, 0, 0, K13_O32, K13_GFP>(a);
}
// (The general path's run mode, fused_device.hpp RT, is a tuner variant: the
// kernel 13 % slower than this one at the level-15 shard length, the pipeline
// line 962 against 1009 GiB/s, profiles/r10e_session.)
__global__ __launch_bounds__(fused::FTPB) void zfec_bao_fused_kernel_general(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, false, 1, 0, 0, true, 1, 0, K13_O32, K13_GFP>(a);
}
__global__ __launch_bounds__(fused::FTPB) void zfec_bao_fused_kernel_full_a64(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, true, 1, 0, 0, true, 0, 0, false, K13_GFP>(a);
}
__global__ __launch_bounds__(fused::FTPB) void zfec_bao_fused_kernel_general_a64(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, false, 1, 0, 0, true, 1, 0, false, K13_GFP>(a);
}
__global__ __launch_bounds__(fused::FTPB) void bao_content_fused_kernel(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, true, 1, 0, 1, true, 0, 0, K13_O32, 0, fused::FW, K13_NTL>(a);
}
__global__ __launch_bounds__(fused::FTPB) void bao_content_fused_kernel_a64(fused::FusedArgs a) {
    fused::zfec_bao_fused_body<true, true, 1, 0, 1>(a);
}

}  // namespace fused

namespace {

// One launch per part of the batch small enough for the kernel's 32-bit block
// queue (< 2^31 blocks; a part is whole objects).  cv_nodes: CVs per object
// the kernel writes into a.cv.
hipError_t launch_parts(const fused::FusedArgs &a, uint64_t cv_nodes, void (*kern)(fused::FusedArgs),
                        hipStream_t stream) {
    using namespace fused;
    const uint64_t per = std::max<uint64_t>(1, (1ull << 31) / std::max<uint64_t>(1, a.bpo));
    for (uint64_t o0 = 0; o0 < a.count; o0 += per) {
        FusedArgs p = a;
        p.count = std::min(per, a.count - o0);
        p.in = a.in + o0 * a.in_stride;
        p.out = a.out + o0 * a.out_stride;
        p.cv = a.cv + o0 * cv_nodes * 32;
        if (a.cv3) p.cv3 = a.cv3 + o0 * a.cvs * 32;
        const uint64_t blocks = p.count * p.bpo;
        uint64_t grid = (blocks + FW - 1) / FW;
        const uint64_t cap = (uint64_t)num_cus();  // one workgroup (8 waves) per CU fits the LDS
        if (grid > cap) grid = cap;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(FTPB), LDS_BYTES, stream, p);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// The tree above the level-3 CVs (cv3 [count][n3]; `spare` holds count *
// ((n3 + 1) / 2) CVs).  Batches of many small trees (>= 2048 objects of 65 to
// 512 level-3 nodes, e.g. 16384 x 1 MiB) run levels 4-6 in the levels pass
// first (one lane per 8 level-3 nodes), so the one-wave-per-object top walk
// starts at level 7 over n3 / 8 nodes instead of walking nine levels from a
// few hundred.  CHIP_UPPER_PASS=0: the walk from level 4 (A/B).
hipError_t upper_levels(uint8_t *cv3, uint64_t n3, uint8_t *spare, uint64_t N, uint64_t count, const uint64_t *coff,
                        uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, hipStream_t stream) {
    static const bool pass_on = [] {
        const char *v = std::getenv("CHIP_UPPER_PASS");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    if (pass_on && count >= 2048 && n3 > 64 && n3 <= (uint64_t)bao::K4T_MAX) {
        const uint64_t n6 = (n3 + 7) / 8, work = count * n6;
        hipLaunchKernelGGL(fused::bao_levels123_lds_kernel<4>, dim3((unsigned)((work + 63) / 64)), dim3(64), 0, stream,
                           cv3, n3, count, coff, d_out, out_stride, spare, n6, (uint64_t)0, (uint64_t)0, (uint64_t)0,
                           (uint32_t)3);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return bao::run_parent_levels<0, false>(spare, n6, n6, 7, cv3, (n6 + 1) / 2, N, count, d_out, out_stride,
                                                d_hash, nullptr, stream);
    }
    return bao::run_parent_levels<0, false>(cv3, n3, n3, 4, spare, (n3 + 1) / 2, N, count, d_out, out_stride, d_hash,
                                            nullptr, stream);
}

}  // namespace

hipError_t zfec_bao_fused_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch,
                              hipStream_t stream) {
    if (count == 0) return hipSuccess;
    if (C == 0 || C % 1024) return hipErrorInvalidValue;
    using namespace fused;
    FusedArgs a{};
    a.in = d_in; a.in_stride = in_stride; a.valid = n; a.C = C;
    a.out = d_out; a.out_stride = out_stride;
    a.count = count;
    a.cols = C / 1024;
    a.N = 8 * a.cols;
    a.bpo = (a.cols + 7) / 8;
    a.cvs = a.N / 8;
    const void *tab = nullptr;
    hipError_t e = zfec_parity_table(4, 8, &tab);
    if (e != hipSuccess) return e;
    a.table = static_cast<const uint32_t *>(tab);
    const uint64_t *coff = nullptr;
    if ((e = bao_chunk_table(a.N, &coff)) != hipSuccess) return e;
    a.coff = coff;
    a.cv = static_cast<uint8_t *>(d_scratch);
    uint32_t *q = nullptr;
    if ((e = stream_queue(stream, &q)) != hipSuccess) return e;
    a.queue = q + QUEUE_K13;
    const bool full = a.cols % 8 == 0 && n >= 4 * C;  // levels 1-3 in the kernel (N >= 64, 8 subtrees a block)
    constexpr auto KF64 = zfec_bao_fused_kernel_full_a64;
    constexpr auto KG64 = zfec_bao_fused_kernel_general_a64;
    constexpr auto KF32 = zfec_bao_fused_kernel_full;
    constexpr auto KG32 = zfec_bao_fused_kernel_general;
    static bool attr = [] {
        bool ok = true;
        for (auto k : {KF64, KG64, KF32, KG32})
            ok &= hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)LDS_BYTES) == hipSuccess;
        return ok;
    }();
    const bool o32 = o32_ok(C);
    const auto KF = o32 ? KF32 : KF64, KG = o32 ? KG32 : KG64;
    (void)attr;
    (void)hipGetLastError();
    const uint64_t n0 = full ? a.N / 8 : a.N;  // nodes per object in `cv`
    uint8_t *next = a.cv + count * n0 * 32;
    if ((e = launch_parts(a, n0, full ? KF : KG, stream)) != hipSuccess) return e;
    if (full) return upper_levels(a.cv, n0, next, a.N, count, coff, d_out, out_stride, d_hash, stream);
    // A tree of at most 8 chunks (C == 1024: N == 8) has its root among
    // levels 1-3; the levels pass would store it as a non-root parent, so the
    // walk runs from level 1 over the chunk CVs and finalizes the root itself.
    if (a.N <= 8)
        return bao::run_parent_levels<0, false>(a.cv, a.N, a.N, 1, next, (a.N + 1) / 2, a.N, count, d_out,
                                                out_stride, d_hash, nullptr, stream);
    // levels 1-3 of every group from the level-0 CVs, then from level 4
    const uint64_t n3 = (a.N + 7) / 8, work = count * n3;
    // a whole level's nodes staged per round (QS 4): node by node (QS 1, 4 KiB
    // of LDS per wave) measured no better (0.391 vs 0.373 ms per 256 objects,
    // tools/fused_tune r10g; pipeline lines equal within noise)
    hipLaunchKernelGGL(fused::bao_levels123_lds_kernel<4>, dim3((unsigned)((work + 63) / 64)), dim3(64), 0, stream,
                       a.cv, a.N, count, coff, d_out, out_stride, next, n3, a.cols, a.bpo, (uint64_t)0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return upper_levels(next, n3, a.cv, a.N, count, coff, d_out, out_stride, d_hash, stream);
}

// Row copy for the device-only levels without a kernel stage (decode at
// Zfec only, encode at level 0): hipMemcpy2DAsync refuses device-to-device
// copies of many-GiB batches ("invalid argument"), so a plain grid-stride
// copy, 16 B per lane (pointers and pitches are multiples of 16 by the
// C-ABI's rules), bytes for a ragged row end.
static __global__ __launch_bounds__(256) void copy_rows_kernel(uint8_t *dst, uint64_t dpitch, const uint8_t *src,
                                                               uint64_t spitch, uint64_t width, uint64_t rows) {
    const uint64_t vec = width / 16, per_row = vec + (width % 16 ? 1 : 0), total = per_row * rows;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = i / per_row, c = i - r * per_row;
        const uint8_t *s = src + r * spitch;
        uint8_t *d = dst + r * dpitch;
        if (c < vec) {
            *reinterpret_cast<uint4 *>(d + 16 * c) = *reinterpret_cast<const uint4 *>(s + 16 * c);
        } else {
            for (uint64_t b = 16 * vec; b < width; ++b) d[b] = s[b];
        }
    }
}

hipError_t copy_rows_dev(uint8_t *dst, uint64_t dpitch, const uint8_t *src, uint64_t spitch, uint64_t width,
                         uint64_t rows, hipStream_t stream) {
    if (!width || !rows) return hipSuccess;
    const uint64_t work = ((width + 15) / 16) * rows;
    uint64_t grid = (work + 255) / 256;
    const uint64_t cap = (uint64_t)num_cus() * 8;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)grid), dim3(256), 0, stream, dst, dpitch, src, spitch, width,
                       rows);
    return hipGetLastError();
}

bool fused_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_FUSED");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

// Content mode: objects of at least one 64-chunk block; whole blocks run in
// KIND 1, the last < 64 chunks (when 64 KiB does not divide n) in the tail
// kernel.
bool bao_fused_ok(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count) {
    return n >= 65536 && (reinterpret_cast<uintptr_t>(d_in) & 15) == 0 && (count <= 1 || in_stride % 16 == 0) &&
           count < (1ull << 31);
}

hipError_t bao_fused_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint8_t *d_out,
                         uint64_t out_stride, uint8_t *d_hash, void *d_scratch, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    if (!bao_fused_ok(d_in, in_stride, n, count)) return hipErrorInvalidValue;
    using namespace fused;
    FusedArgs a{};
    a.in = d_in; a.in_stride = in_stride; a.valid = n; a.C = 0;
    a.out = d_out; a.out_stride = out_stride;
    a.count = count;
    a.N = bao::n_chunks(n);
    a.cols = 0;
    a.bpo = n / 65536;                 // whole 64-chunk blocks (every chunk 1 KiB)
    a.cvs = (a.N + 7) / 8;             // level-3 CVs per object
    const uint64_t Nf = 64 * a.bpo;    // chunks [Nf, N): the tail kernel
    a.table = nullptr;
    const uint64_t *coff = nullptr;
    hipError_t e = bao_chunk_table(a.N, &coff);
    if (e != hipSuccess) return e;
    a.coff = coff;
    a.cv = static_cast<uint8_t *>(d_scratch);
    uint32_t *q = nullptr;
    if ((e = stream_queue(stream, &q)) != hipSuccess) return e;
    a.queue = q + QUEUE_K13;
    constexpr auto K64 = bao_content_fused_kernel_a64;
    constexpr auto K32 = bao_content_fused_kernel;
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(K64), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)LDS_BYTES) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void *>(K32), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)LDS_BYTES) == hipSuccess;
    }();
    const auto K = o32_ok(n) ? K32 : K64;
    (void)attr;
    (void)hipGetLastError();
    const uint64_t n3 = a.cvs;
    if ((e = launch_parts(a, n3, K, stream)) != hipSuccess) return e;
    if (Nf < a.N) {
        TailArgs t{};
        t.in = d_in; t.in_stride = in_stride; t.n = n;
        t.out = d_out; t.out_stride = out_stride;
        t.count = count; t.N = a.N; t.Nf = Nf; t.cvs = n3;
        t.coff = coff; t.cv = a.cv;
        hipLaunchKernelGGL(bao_tail_kernel, dim3((unsigned)count), dim3(64), 0, stream, t);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    uint8_t *next = a.cv + count * n3 * 32;
    return upper_levels(a.cv, n3, next, a.N, count, coff, d_out, out_stride, d_hash, stream);
}

}  // namespace chip
