// chip_internal.hpp — shared declarations of libcarbonado_hip (gfx950).
//
// Layering:
//   gf256.hpp            host GF(2^8) arithmetic: zfec matrices, inverses,
//                        packed LDS tables (built once per (k, m, pattern))
//   zfec_kernels.hip     K1/K2: GF(2^8) stripe matrix-apply (encode and
//                        erasure decode are the same kernel)
//   bao_kernels.hip      K3/K4/K5: BLAKE3 chunk CVs, parent levels, bao
//                        pre-order layout, verify-decode
//   fused_kernels.hip    K13: zfec + bao in one pass; content-mode bao
//   api_*.cpp            the C-ABI (include/carbonado_hip.h): host staging,
//                        per-thread streams, error mapping, pipeline glue
//                        (api_common.hpp lists the files by concern)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstddef>
#include <vector>

#include "../../include/carbonado_hip.h"

namespace chip {

constexpr uint64_t NO_OUT = ~0ull;
constexpr int ZF_MAXK = 16;  // fast kernel: up to 16 input shards
constexpr int ZF_MAXP = 8;   // fast kernel: up to 8 computed rows (2 dword groups)

// One GF(2^8) "matrix apply" over stripes of `count` objects:
//   out_row[p] = XOR_j coef[p][j] * in_row[j]    (computed rows)
//   out_row    = in_row[j]                       (copy rows, copy_off[j])
// Encode: in rows = the k data shards (zero beyond `valid`), copies = data
// shards, computed rows = parity.  Decode: in rows = k surviving shares,
// copies = surviving primaries, computed rows = the lost primaries.
struct GfPlan {
    uint32_t k = 0;                 // input rows
    uint32_t np = 0;                // computed rows
    uint64_t in_off[ZF_MAXK];       // offset of input row j inside an input object
    uint64_t copy_off[ZF_MAXK];     // output offset for a copy of input row j, or NO_OUT
    std::vector<uint64_t> comp_off; // output offset of each computed row (np)
    std::vector<uint8_t> coef;      // np x k
    // generic path (k > 16 or np > 8): full row lists
    std::vector<uint64_t> g_in_off;   // k
    std::vector<uint64_t> g_out_off;  // rows
    std::vector<uint8_t> g_coef;      // rows x k (copies expressed as unit rows)
};

struct GfLaunch {
    const uint8_t *in;
    uint8_t *out;
    uint64_t in_stride, out_stride;
    uint64_t valid;   // bytes of each input object that are data (rest reads as 0)
    uint64_t C;       // shard length (multiple of 16)
    uint64_t count;   // objects
    // optional: write the shard-major output in bao layout (encode() with
    // Zfec|Bao): stream offset of each 1 KiB content chunk, device table
    const uint64_t *bao_off = nullptr;
    // optional: at most this many workgroups per CU (0 = occupancy), leaving
    // room for a kernel that runs beside it on another stream
    int wg_per_cu = 0;
    // diagnostic (chip_hbm_pattern_batch_dev): the same launch with the GF
    // arithmetic taken out — the bare memory pattern the kernel is priced by
    bool pattern_only = false;
};

// Enqueue the matrix apply.  Tables are cached device-side per plan key.
// Plans with more than ZF_MAXP computed rows run in passes of ZF_MAXP rows
// (copies ride on the first pass); k outside the fast kernel's instances (1..8,
// 16) uses the generic kernel.
hipError_t gf_apply(const GfPlan &plan, const GfLaunch &L, hipStream_t stream);
// Device copy of the packed parity table of a k-of-m encode (m - k <= 4):
// [k][256] dwords, byte r of entry [s][x] = E[k + r][s] * x (cached).
hipError_t zfec_parity_table(uint32_t k, uint32_t m, const void **out);
// Per-stream block of zeroed run-queue counters (4 KiB) shared by the
// persistent kernels launched on that stream: K1 words 0-256, K13 from word
// QUEUE_K13, K3 from word QUEUE_K3 (two counters 32 words apart each).
constexpr int QUEUE_K13 = 512;
constexpr int QUEUE_K3 = 640;
constexpr int QUEUE_KM = 768;  // KM's last-workgroup counter
hipError_t stream_queue(hipStream_t stream, uint32_t **out);
// Return a stream's block to the pool; call once the stream's work is done,
// before the stream is destroyed (a later stream may get the same handle).
void stream_queue_release(hipStream_t stream);

// ---- K13: encode() at Zfec|Bao in one pass (fused_kernels.hip) ----------
// `count` objects of n bytes (zero padded to 4C) -> bao streams of their
// 4-of-8 zfec outputs (8C bytes each) + root hashes; scratch of
// zfec_bao_scratch_len(8C, count) bytes (level-0 CVs + one tree level).
uint64_t zfec_bao_scratch_len(uint64_t zlen, uint64_t count);
hipError_t zfec_bao_fused_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch,
                              hipStream_t stream);

// The same kernel for bao of the content itself (encoding::bao, encode() at
// the Bao bit, level 4) for n >= 64 KiB with 16-B aligned rows: the whole
// 64-chunk blocks in KIND 1, the rest in bao_tail_kernel; bao_encode_dev takes
// it then.  Scratch: bao_scratch_len covers it.
bool bao_fused_ok(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count);
hipError_t bao_fused_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint8_t *d_out,
                         uint64_t out_stride, uint8_t *d_hash, void *d_scratch, hipStream_t stream);
// CHIP_FUSED (default 1): 0 keeps the two-kernel / K3 paths (A/B runs).
bool fused_on();
// `rows` rows of `width` bytes, device to device (16-B aligned pointers/pitches).
hipError_t copy_rows_dev(uint8_t *dst, uint64_t dpitch, const uint8_t *src, uint64_t spitch, uint64_t width,
                         uint64_t rows, hipStream_t stream);

// ---- bao / BLAKE3 ------------------------------------------------------
uint64_t bao_encoded_len(uint64_t n);
uint64_t bao_scratch_len(uint64_t n, uint64_t count);
// Encode `count` objects of n bytes; hashes to d_hash (32 B each).
hipError_t bao_encode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                          uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch,
                          hipStream_t stream);
// Verify-decode; d_status[o] = 0 or CHIP_ERR_BAO_HASH_MISMATCH.
hipError_t bao_decode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                          const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride,
                          uint32_t *d_status, void *d_scratch, hipStream_t stream);
// The same, writing only content bytes [0, out_limit) of each object (every
// byte is still verified): decode() at Bao|Zfec keeps the data shards only.
hipError_t bao_decode_prefix_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                                 const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride, uint64_t out_limit,
                                 uint32_t *d_status, void *d_scratch, hipStream_t stream);

// bao encode in place: the stream's chunk slots already hold the content
// (written there by gf_apply with GfLaunch::bao_off); writes the header, the
// parent nodes and the hashes.
hipError_t bao_encode_inplace_dev(uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count, uint8_t *d_hash,
                                  void *d_scratch, hipStream_t stream);
// Cached device table [N] of the stream offsets of the N content chunks.
hipError_t bao_chunk_table(uint64_t N, const uint64_t **out);

// Per-node bao verification (K5b): chunk_flags [count][N], parent_flags
// [count][N-1] in stream order; 1 = the node matches the copy stored in its
// parent (the root: the hash).
hipError_t bao_node_check(const uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count,
                          const uint8_t *d_hash, uint8_t *chunk_flags, uint8_t *parent_flags, hipStream_t stream);
// scrub(): per-object mask of authentic zfec shards (bit i = shard i) of
// Bao|Zfec streams from bao_node_check's flags; spc = chunks per shard.
hipError_t scrub_masks(const uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count, uint64_t spc,
                       const uint8_t *chunk_flags, const uint8_t *parent_flags, uint8_t *masks, hipStream_t stream);
// Content of chunks [c0, c1) of one stream, parents stripped, to d_out.
hipError_t bao_gather_content(const uint8_t *d_stream, uint64_t n, uint64_t c0, uint64_t c1, uint8_t *d_out,
                              hipStream_t stream);
// Incremental BaoHasher: chunk CVs of full, non-final chunks [c0, c1) of a
// contiguous content buffer (cv0[i] = chunk i's CV, 32 B); at finalize the
// remaining chunks [c_done, N), the content laid out in the stream d_out,
// the parent levels (cv0 and cv1 ((N+1)/2 CVs) as ping-pong buffers, cv0
// overwritten) and the root hash.  N = n_chunks(n) must be >= 2.
hipError_t hasher_chunks_dev(const uint8_t *content, uint64_t n, uint64_t c0, uint64_t c1, uint8_t *cv0,
                             hipStream_t stream);
hipError_t hasher_finish_dev(const uint8_t *content, uint64_t n, uint64_t c_done, uint8_t *cv0, uint8_t *cv1,
                             uint8_t *d_out, uint8_t *d_hash, hipStream_t stream);
// The parent nodes in front of chunks [0, nd) of `count` streams of N chunks
// (their data region when the content is a zfec output: nd = N/2), in stream
// order, to d_nodes (nodes_stride >= 64 * bao_data_node_count(N, nd), both
// strides multiples of 8).
uint64_t bao_data_node_count(uint64_t N, uint64_t nd);
hipError_t bao_data_nodes(const uint8_t *d_stream, uint64_t stride, uint64_t N, uint64_t nd, uint64_t count,
                          uint8_t *d_nodes, uint64_t nodes_stride, hipStream_t stream);
// Content bytes [0, nbytes) of `count` streams of N chunks from their chunk
// slots to contiguous rows (nbytes <= 1024 N; strides multiples of 8).
hipError_t bao_gather_rows(const uint8_t *d_stream, uint64_t stride, uint64_t N, uint64_t count, uint64_t nbytes,
                           uint8_t *d_out, uint64_t out_stride, hipStream_t stream);
// Stream layout (host side, same formulas as the kernels).
uint64_t bao_chunk_offset(uint64_t i, uint64_t N);
uint64_t bao_parent_offset(uint64_t s, int level, uint64_t N);
uint64_t bao_parent_index(uint64_t s, int level, uint64_t N);

// ---- KS: small objects, one workgroup per object (small_kernels.hip) ----
// Latency path for count == 1 and a bao stream of at most KS_MAX_N chunks,
// and the batch path for tiny objects (at most KS_TINY_N chunks, one wave
// each); CHIP_SMALL=0 turns both off.  The batch entry points take them
// themselves when small_ok() holds.
// tiny_max: the largest N for which the caller's batch kernel loses to KS
// (measured per path, DESIGN.md §3 KS; at most KS_TINY_N).
constexpr uint64_t KS_MAX_N = 512;
constexpr uint64_t KS_TINY_N = 64;
bool small_ok(uint64_t bao_n, uint64_t count, uint64_t tiny_max = KS_TINY_N);
hipError_t small_bao_encode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                                uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, hipStream_t stream);
hipError_t small_zfec_bao_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, hipStream_t stream);
hipError_t small_bao_decode_dev(const uint8_t *d_stream, uint64_t in_stride, uint64_t n, uint64_t count,
                                const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride, uint64_t out_limit,
                                uint32_t *d_status, hipStream_t stream);

// ---- KM: one single object over many workgroups (multi_kernels.hip) ----
// Latency path for count == 1 and a bao stream of KS_TINY_N < N <= KM_MAX_N
// chunks: a quad of lanes per compression, a 64-chunk subtree per workgroup,
// the last workgroup to finish walks the tree top (CHIP_KM=0 turns it off).
// Scratch: km_scratch_len(bao_n) bytes (the group CVs).
constexpr uint64_t KM_MAX_N = 32768;
bool km_ok(uint64_t bao_n, uint64_t count);
// one object from host memory on the zero-copy single-object paths
// (api_single.cpp): KM for 64 < N <= KM_MAX_N, KS up to 64 chunks (n > 0)
bool single_ok(uint64_t bao_n);
bool km_enabled();  // CHIP_KM (default on): also the single-object zero-copy zfec encode
// the single-object zero-copy zfec paths (api_single.cpp) for a pinned
// footprint of `bytes`: km_enabled() and at most ZC_MAX_BYTES (larger objects
// take the staged copies through the 16 MiB ring instead of pinning their size)
constexpr uint64_t ZC_MAX_BYTES = uint64_t(64) << 20;
inline bool zc_ok(uint64_t bytes) { return bytes <= ZC_MAX_BYTES && km_enabled(); }
uint64_t km_scratch_len(uint64_t bao_n);
// bao of n content bytes at d_in (device or pinned host memory): the parent
// nodes compactly into d_nodes (the node at stream offset o in front of chunk
// s goes to o - 8 - 1024 s; null: none), the root hash to d_hash.
hipError_t km_bao_encode_dev(const uint8_t *d_in, uint64_t n, uint8_t *d_nodes, uint8_t *d_hash, void *d_scratch,
                             hipStream_t stream);
// encode() at Zfec|Bao of `valid` input bytes at d_in (16-B aligned, zero
// padded to 4 C by the masked loads): the 8 shards into the chunk slots of
// d_stream (device), the parity shards and the nodes past the data region
// also into d_tail = the stream's image from byte t0 (null: none), the nodes
// of the data region (chunks [0, 4 C / 1024)) compactly into d_nodes as
// above, the hash.  parity_done (optional) is recorded once the shards are
// written (d_tail's chunks final; the nodes follow with KM).
hipError_t km_zfec_bao_dev(const uint8_t *d_in, uint64_t valid, uint64_t C, uint8_t *d_stream, uint8_t *d_nodes,
                           uint8_t *d_tail, uint64_t t0, uint8_t *d_hash, void *d_scratch, hipStream_t stream,
                           hipEvent_t parity_done = nullptr);
// encoding::zfec 4-of-8 of `valid` input bytes at d_in (pinned host or
// device memory, 16-B aligned): the 4 parity shards, shard-major, to d_par.
hipError_t zc_zfec_parity_dev(const uint8_t *d_in, uint64_t valid, uint64_t C, uint8_t *d_par, hipStream_t stream);
// verify-decode one stream of n content bytes; content [0, out_limit) to
// d_out (null: verify only); d_status (zero at launch) = 0 or
// CHIP_ERR_BAO_HASH_MISMATCH.
hipError_t km_bao_decode_dev(const uint8_t *d_stream, uint64_t n, const uint8_t *d_hash, uint8_t *d_out,
                             uint64_t out_limit, uint32_t *d_status, void *d_scratch, hipStream_t stream);

// ---- batch buffers (hbm_alloc.hip) --------------------------------------
// Class-balanced device memory for buffers >= 1 GiB (hbm_alloc.hpp); returns
// an error for smaller sizes or when the virtual-memory API fails.
hipError_t hbm_alloc(uint64_t bytes, void **out);
bool hbm_free(void *p);  // true if p came from hbm_alloc
bool hbm_info(const void *p, uint32_t *classes_found, uint32_t *classes_used, double *seconds);

// ---- context ------------------------------------------------------------
int ensure_device();                 // CHIP_OK or CHIP_ERR_NO_DEVICE
int use_device();                    // ensure_device() + make the process's device current
int selected_device();               // the process's device (chip_init / default)
void set_device_error(hipError_t e); // remember for chip_last_device_error
int num_cus();

}  // namespace chip
