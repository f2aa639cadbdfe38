// bao_kernels.hip — K3/K4/K5 host side: BLAKE3 chunk chaining values, parent
// levels and the bao combined (pre-order) layout on gfx950.
//
// Replaces bao 0.12.1 -> blake3 1.x as called from
//   encoding::bao  /root/reference/src/encoding.rs:38-44  (bao::encode::encode)
//   decoding::bao  /root/reference/src/decoding.rs:53-60  (bao::decode::decode)
//
// Layout facts used (BLAKE3 spec; bao combined encoding):
//   * content is cut into N = max(1, ceil(n/1024)) chunks; chunk i is hashed
//     with counter i in 64-byte blocks (CHUNK_START on block 0, CHUNK_END on
//     the last, ROOT on the last block iff N == 1);
//   * the tree is the left-to-right pairwise merge of each level, an odd last
//     node promoted unchanged (== "left subtree = largest power of two");
//   * the stream is u64 LE n, then pre-order: each parent's 64 bytes
//     (left CV || right CV) precede its subtrees.  With c(s) = number of
//     parents whose leftmost chunk is s (= min(tz(s), ceil_log2(N-s)),
//     ceil_log2(N) for s = 0) and P(s) = sum_{j<s} c(j):
//         chunk i           at 8 + 1024 i + 64 (P(i) + c(i))
//         parent (level l, first chunk s) at 8 + 1024 s + 64 (P(s) + c(s) - l)
//
// K3 (bao_chunk_kernel, bao_device.hpp): lane = CPL consecutive chunks, the
// first log2(CPL) levels folded in registers; chunk bytes staged through LDS
// once and written straight to their stream slot (encode) or content slot
// (decode).  BLAKE3 is VALU work (672 lane-ops per 64-B block): hash-only K3
// is VALU-bound; with the stream written, the store pattern costs ~40 %.
// Encode keeps two steps per LDS row (SP 3) so every 128-B stream line is
// stored whole; CPL 2 keeps a wave's 64 write fronts within 128 KiB.
// K4 (bao_parent_kernel): one launch per remaining level, lane = one node.
// K5 (verify-decode) = the same kernels in MODE 1: every stored parent node is
// compared with the recomputed children, the root with the expected hash.
#include "bao_device.hpp"
#include "chip_internal.hpp"

#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

namespace chip {

using namespace bao;

namespace {

// tuned on MI355X (tools/bao_tune.hip): CPL 8 / SP 0 1.38 TiB/s,
// CPL 4 / SP 3 1.49, CPL 2 / SP 3 1.58 (encode with stream, 256 x 32 MiB);
// decode CPL 2 1.88 vs CPL 8 1.77.
constexpr int BAO_CPL = 2;
constexpr bool BAO_NTS = false;
// Verify-decode writes the content in whole 128-B lines it never reads back:
// nontemporal, or the L2 fetches every destination line first (PMC: reads
// 1.59x the stream with plain stores, r2q_baodec_pmc.json; tools/fetch_calib
// pins FETCH_SIZE at 1/2 of the bytes for these loads).
#ifndef BAO_DEC_NTS_DEF
#define BAO_DEC_NTS_DEF true
#endif
constexpr bool BAO_DEC_NTS = BAO_DEC_NTS_DEF;
constexpr int BAO_SP = 3;
// XCD-grouped block order: +0.9-1.8 % on encode / decode / in-place (tools/bao_tune, r1x)
constexpr int BAO_XG = 1;
// SP 3 store loop fully unrolled over the 8 chunk groups: +0.6-0.9 % (tools/bao_tune, r1x)
constexpr int BAO_SU = 8;
// Persistent grid with wave tasks from the stream's run queue: the XCDs do
// not stream at one rate, and a static grid ends on the slowest (K13 measured
// +5.6-7.8 % from the same change, tools/fused_tune r2l).
constexpr bool BAO_DQ = true;

}  // namespace

// The product's K3 configurations, one kernel each (bao_device.hpp ChunkKernel):
// encode (MODE 0, the stream written), verify-decode (MODE 1, the content
// written, whole or a prefix), node check (MODE 2, scrub), in-place encode
// (MODE 3, the two-kernel Zfec|Bao path); _static: without the run queue (a
// batch of 2^31 wave tasks or more).
#define CHIP_K3(NAME, MODE, CPL, NTS, SP, SU)                                                   \
    __global__ __launch_bounds__(K3_TPB) void NAME(ChunkArgs a) {                              \
        bao_chunk_body<MODE, CPL, NTS, SP, SU, 0, BAO_XG, BAO_DQ>(a);                          \
    }                                                                                         \
    __global__ __launch_bounds__(K3_TPB) void NAME##_static(ChunkArgs a) {                     \
        bao_chunk_body<MODE, CPL, NTS, SP, SU, 0, BAO_XG, false>(a);                           \
    }                                                                                         \
    template <>                                                                               \
    struct ChunkKernel<MODE, CPL, NTS, SP, SU, 0, BAO_XG, true> {                             \
        static constexpr void (*fn)(ChunkArgs) = NAME;                                        \
    };                                                                                        \
    template <>                                                                               \
    struct ChunkKernel<MODE, CPL, NTS, SP, SU, 0, BAO_XG, false> {                            \
        static constexpr void (*fn)(ChunkArgs) = NAME##_static;                               \
    };
namespace bao {
CHIP_K3(bao_chunk_kernel_encode, 0, BAO_CPL, BAO_NTS, BAO_SP, BAO_SU)
CHIP_K3(bao_chunk_kernel_verify, 1, BAO_CPL, BAO_DEC_NTS, 0, 1)
CHIP_K3(bao_chunk_kernel_check, 2, 1, false, 0, 1)
CHIP_K3(bao_chunk_kernel_inplace, 3, 8, BAO_NTS, 0, 1)
}  // namespace bao
#undef CHIP_K3

namespace {

template <int MODE>
hipError_t run_bao(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                   uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, uint32_t *d_status,
                   void *d_scratch, hipStream_t stream) {
    return run_bao_t<MODE, BAO_CPL, MODE == 1 ? BAO_DEC_NTS : BAO_NTS, MODE == 0 ? BAO_SP : 0, MODE == 0 ? BAO_SU : 1, 0,
                     BAO_XG, BAO_DQ>(
        d_in, in_stride, n, count, d_out, out_stride, d_hash, d_status, d_scratch, stream);
}

}  // namespace

uint64_t bao_encoded_len(uint64_t n) { return 8 + n + 64 * (n_chunks(n) - 1); }

uint64_t bao_scratch_len(uint64_t n, uint64_t count) { return bao_scratch_len_t<BAO_CPL>(n, count); }

hipError_t bao_encode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                          uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch,
                          hipStream_t stream) {
    // batches: KS below 64 KiB, where K13's content mode cannot take whole 64-chunk blocks
    // (r4q: 32 KiB objects 1032 vs 528 GiB/s; 64 KiB: K13 1477 vs KS 1046)
    const bool k13 = d_out && fused_on() && bao_fused_ok(d_in, in_stride, n, count);
    if (small_ok(n, count, k13 ? 0 : KS_TINY_N))
        return small_bao_encode_dev(d_in, in_stride, n, count, d_out, out_stride, d_hash, stream);
    if (k13)  // K13 KIND 1 (fused_kernels.hip)
        return bao_fused_dev(d_in, in_stride, n, count, d_out, out_stride, d_hash, d_scratch, stream);
    return run_bao<0>(d_in, in_stride, n, count, d_out, out_stride, d_hash, nullptr, d_scratch, stream);
}

hipError_t bao_decode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                          const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride,
                          uint32_t *d_status, void *d_scratch, hipStream_t stream) {
    if (small_ok(n, count))
        return small_bao_decode_dev(d_in, in_stride, n, count, d_hash, d_out, out_stride, n, d_status, stream);
    return run_bao<1>(d_in, in_stride, n, count, d_out, out_stride, const_cast<uint8_t *>(d_hash),
                      d_status, d_scratch, stream);
}

hipError_t bao_decode_prefix_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                                 const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride, uint64_t out_limit,
                                 uint32_t *d_status, void *d_scratch, hipStream_t stream) {
    if (small_ok(n, count))
        return small_bao_decode_dev(d_in, in_stride, n, count, d_hash, d_out, out_stride, std::min(out_limit, n),
                                    d_status, stream);
    return run_bao_t<1, BAO_CPL, BAO_DEC_NTS, 0, 1, 0, BAO_XG, BAO_DQ>(d_in, in_stride, n, count, d_out, out_stride,
                                                          const_cast<uint8_t *>(d_hash), d_status, d_scratch, stream,
                                                          0, out_limit);
}

hipError_t bao_node_check(const uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count,
                          const uint8_t *d_hash, uint8_t *chunk_flags, uint8_t *parent_flags, hipStream_t stream) {
    return run_node_check(d_stream, stride, n, count, d_hash, chunk_flags, parent_flags, stream);
}

hipError_t bao_gather_content(const uint8_t *d_stream, uint64_t n, uint64_t c0, uint64_t c1, uint8_t *d_out,
                              hipStream_t stream) {
    const uint64_t N = n_chunks(n);
    if (c1 > N) c1 = N;
    if (c0 >= c1 || c0 * 1024 >= n) return hipSuccess;
    const uint64_t bytes = (c1 * 1024 < n ? c1 * 1024 : n) - c0 * 1024;
    uint64_t blocks = (bytes / 16 + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
    hipLaunchKernelGGL(bao_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_stream, n, N, c0, c1, d_out);
    return hipGetLastError();
}

uint64_t bao_data_node_count(uint64_t N, uint64_t nd) {
    return nd ? (chunk_stream_off(nd - 1, N) + 1024 - 8 - 1024 * nd) / 64 : 0;
}

hipError_t bao_data_nodes(const uint8_t *d_stream, uint64_t stride, uint64_t N, uint64_t nd, uint64_t count,
                          uint8_t *d_nodes, uint64_t nodes_stride, hipStream_t stream) {
    if (!nd || !count) return hipSuccess;
    if (nd > N || (stride % 8) || (nodes_stride % 8) || nodes_stride < 64 * bao_data_node_count(N, nd))
        return hipErrorInvalidValue;
    const uint64_t *coff = nullptr;
    hipError_t e = bao_chunk_table(N, &coff);
    if (e != hipSuccess) return e;
    uint64_t blocks = (count * nd * 8 + 255) / 256;
    blocks = blocks > 16384 ? 16384 : blocks;
    hipLaunchKernelGGL(bao_data_nodes_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_stream, stride, coff,
                       nd, count, d_nodes, nodes_stride);
    return hipGetLastError();
}

hipError_t bao_gather_rows(const uint8_t *d_stream, uint64_t stride, uint64_t N, uint64_t count, uint64_t nbytes,
                           uint8_t *d_out, uint64_t out_stride, hipStream_t stream) {
    if (!count || !nbytes) return hipSuccess;
    if (nbytes > 1024 * N || (stride % 8) || (out_stride % 8) || out_stride < nbytes) return hipErrorInvalidValue;
    const uint64_t *coff = nullptr;
    hipError_t e = bao_chunk_table(N, &coff);
    if (e != hipSuccess) return e;
    uint64_t blocks = (count * ((nbytes + 7) / 8) + 255) / 256;
    blocks = blocks > 16384 ? 16384 : blocks;
    hipLaunchKernelGGL(bao_gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_stream, stride, coff,
                       count, nbytes, d_out, out_stride);
    return hipGetLastError();
}

hipError_t bao_encode_inplace_dev(uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count, uint8_t *d_hash,
                                  void *d_scratch, hipStream_t stream) {
    // CPL 8: no content stores here, so the wider lane span costs nothing and
    // three tree levels fold in registers (tools/bao_tune: 3.15 vs 3.39 ms
    // for CPL 2 on 256 x 32 MiB; fewer K4 launches).  Scratch sized for
    // BAO_CPL covers it (N/8 <= N/2 level nodes).
    return run_bao_t<3, 8, BAO_NTS, 0, 1, 0, BAO_XG, BAO_DQ>(d_stream, stride, n, count, d_stream, stride, d_hash,
                                                             nullptr, d_scratch, stream);
}

namespace {
std::mutex g_tab_mu;
std::map<std::pair<int, uint64_t>, uint64_t *> g_chunk_tabs;  // (device, N) -> table [N] of chunk stream offsets
}  // namespace

hipError_t bao_chunk_table(uint64_t N, const uint64_t **out) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    const std::pair<int, uint64_t> key(selected_device(), N);
    auto it = g_chunk_tabs.find(key);
    if (it != g_chunk_tabs.end()) { *out = it->second; return hipSuccess; }
    std::vector<uint64_t> h(N);
    uint64_t off = chunk_stream_off(0, N);
    for (uint64_t i = 0; i < N; ++i) {  // P and c advance incrementally: 1024 + 64 c(i) per chunk
        if (i) off += 1024 + 64 * (uint64_t)parents_at(i, N);
        h[i] = off;
    }
    uint64_t *d = nullptr;
    hipError_t e = hipMalloc(&d, N * 8);
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, h.data(), N * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(d); return e; }
    g_chunk_tabs[key] = d;
    *out = d;
    return hipSuccess;
}

namespace {

// Which of the 8 zfec shards of a Bao|Zfec stream scrub() may use
// (decoding.rs:172-183: verify_slice of each shard's chunk range), from the
// per-node flags of bao_node_check: shard i is authentic iff every chunk in
// its range and every parent whose subtree meets the range verified (the
// nodes bao's slice decoder walks; a parent node is checked against the CV
// stored in its own parent, the root against the hash).  One workgroup per
// object; mask bit i = shard i authentic, 0 for a stream whose header does not
// hold n.
__global__ __launch_bounds__(256) void scrub_mask_kernel(const uint8_t *stream, uint64_t stride, uint64_t n,
                                                         uint64_t N, uint64_t spc, const uint8_t *cflags,
                                                         const uint8_t *pflags, uint8_t *masks) {
    __shared__ uint32_t bad;
    const uint64_t obj = blockIdx.x;
    if (threadIdx.x == 0) bad = *reinterpret_cast<const uint64_t *>(stream + obj * stride) != n ? 0xFFu : 0u;
    __syncthreads();
    uint32_t mine = 0;
    const uint8_t *cf = cflags + obj * N, *pf = pflags + obj * (N - 1);
    for (uint64_t c = threadIdx.x; c < N; c += 256)
        if (!cf[c]) mine |= 1u << (c / spc);
    for (uint64_t r0 = threadIdx.x; r0 + 1 < N; r0 += 256) {  // the r0-th real parent in level order
        uint64_t r = r0, cnt = N;
        int level = 1;
        for (;; ++level) {
            const uint64_t np = cnt / 2;
            if (r < np) break;
            r -= np;
            cnt = (cnt + 1) / 2;
        }
        const uint64_t sx = r << level;
        if (pf[parents_before(sx, N) + parents_at(sx, N) - level]) continue;
        const uint64_t end = sx + (1ull << level) < N ? sx + (1ull << level) : N;
        for (uint64_t sh = sx / spc; sh <= (end - 1) / spc; ++sh) mine |= 1u << sh;
    }
    if (mine) atomicOr(&bad, mine);
    __syncthreads();
    if (threadIdx.x == 0) masks[obj] = (uint8_t)(~bad & 0xFFu);
}

}  // namespace

hipError_t scrub_masks(const uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count, uint64_t spc,
                       const uint8_t *chunk_flags, const uint8_t *parent_flags, uint8_t *masks, hipStream_t stream) {
    const uint64_t N = n_chunks(n);
    if (count == 0) return hipSuccess;
    if (N < 2 || spc == 0 || N != 8 * spc) return hipErrorInvalidValue;
    hipLaunchKernelGGL(scrub_mask_kernel, dim3((unsigned)count), dim3(256), 0, stream, d_stream, stride, n, N, spc,
                       chunk_flags, parent_flags, masks);
    return hipGetLastError();
}

// ---- incremental BaoHasher (utils.rs:104-137) ------------------------------
//
// bao's Encoder takes the content in appends; the chunk CVs of a chunk do not
// depend on what follows it (counter = chunk index, CHUNK_START / CHUNK_END
// on its first / last block, ROOT only when N == 1).  So chunk_update hashes
// chunks as soon as bytes past them have arrived (they are full and not the
// root), and finalize only hashes the last < 64 + 1 chunks, lays the content
// out in its chunk slots and builds the parent levels from the chunk CVs (the
// slot offsets depend on the final N, so the layout waits for it).

namespace {

// chunk CVs of chunks [c0, c1) of a content buffer of n bytes (N > 1: none is
// the root), one lane per chunk
__global__ __launch_bounds__(64) void hasher_chunk_kernel(const uint8_t *content, uint64_t n, uint64_t c0,
                                                          uint64_t c1, uint8_t *cv) {
    const uint64_t ci = c0 + (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (ci >= c1) return;
    const uint8_t *src = content + ci * 1024;
    const uint64_t rem = n - ci * 1024;
    const uint32_t clen = rem < 1024 ? (uint32_t)rem : 1024u;
    const uint32_t nb = clen ? (clen + 63) / 64 : 1;
    uint32_t h[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) h[w] = IV(w);
    for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t blen = clen - 64 * b < 64 ? clen - 64 * b : 64u;
        uint32_t m[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t off = 64 * b + 16 * q;
            const uint32_t valid = off < clen ? clen - off : 0u;
            const u32x4 x = valid >= 16 ? *reinterpret_cast<const u32x4 *>(src + off) : load16_partial(src + off, valid);
            m[4 * q] = x.x; m[4 * q + 1] = x.y; m[4 * q + 2] = x.z; m[4 * q + 3] = x.w;
        }
        const uint32_t flags = (b == 0 ? F_CHUNK_START : 0u) | (b + 1 == nb ? F_CHUNK_END : 0u);
        b3_compress(h, m, ci, blen, flags);
    }
    store_cv(cv + ci * 32, h);
}

// the stream's header and every chunk's content at its slot (one wave per
// chunk, 16 B per lane; slots are 8-B aligned)
__global__ __launch_bounds__(256) void hasher_layout_kernel(const uint8_t *content, uint64_t n, uint64_t N,
                                                            uint8_t *out) {
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) *glb(reinterpret_cast<uint64_t *>(out)) = n;
    for (uint64_t ci = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); ci < N; ci += (uint64_t)gridDim.x * 4) {
        const uint64_t off = chunk_stream_off(ci, N);
        const uint64_t b = ci * 1024 + 16 * (uint64_t)lane;
        if (b + 16 <= n) {
            store16_a8<false>(out + off + 16 * lane, *reinterpret_cast<const u32x4 *>(content + b));
        } else if (b < n) {
            store16_partial(out + off + 16 * lane, load16_partial(content + b, (uint32_t)(n - b)), (uint32_t)(n - b));
        }
    }
}

}  // namespace

hipError_t hasher_chunks_dev(const uint8_t *content, uint64_t n, uint64_t c0, uint64_t c1, uint8_t *cv0,
                             hipStream_t stream) {
    if (c1 <= c0) return hipSuccess;
    const uint64_t blocks = (c1 - c0 + 63) / 64;
    hipLaunchKernelGGL(hasher_chunk_kernel, dim3((unsigned)blocks), dim3(64), 0, stream, content, n, c0, c1, cv0);
    return hipGetLastError();
}

hipError_t hasher_finish_dev(const uint8_t *content, uint64_t n, uint64_t c_done, uint8_t *cv0, uint8_t *cv1,
                             uint8_t *d_out, uint8_t *d_hash, hipStream_t stream) {
    const uint64_t N = n_chunks(n);
    if (N < 2) return hipErrorInvalidValue;  // the single chunk is the root: the batch path
    hipError_t e = hasher_chunks_dev(content, n, c_done, N, cv0, stream);
    if (e != hipSuccess) return e;
    const uint64_t blocks = std::min<uint64_t>((N + 3) / 4, 65536);
    hipLaunchKernelGGL(hasher_layout_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, content, n, N, d_out);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return run_parent_levels<0, false>(cv0, N, N, 1, cv1, (N + 1) / 2, N, 1, d_out, 0, d_hash, nullptr, stream);
}

uint64_t bao_chunk_offset(uint64_t i, uint64_t N) { return chunk_stream_off(i, N); }
uint64_t bao_parent_offset(uint64_t s, int level, uint64_t N) { return parent_stream_off(s, level, N); }
uint64_t bao_parent_index(uint64_t s, int level, uint64_t N) {
    return parents_before(s, N) + parents_at(s, N) - level;
}

}  // namespace chip
