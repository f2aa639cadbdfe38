/*
 * carbonado_hip.h — C-ABI of libcarbonado_hip.so, the MI355X (gfx950) hot
 * path of carbonado's encode()/decode(): zfec k-of-m Reed-Solomon erasure
 * coding over GF(2^8) and bao/BLAKE3 verifiable-stream encoding.
 *
 * Drop-in boundary.  carbonado 0.6.0 routes its hot path through five
 * crate-internal stage functions; each entry point
 * below replaces exactly one of them (citations are /root/reference paths):
 *
 *   chip_zfec_encode        <- encoding::zfec        src/encoding.rs:46-81
 *   chip_bao_encode         <- encoding::bao         src/encoding.rs:38-44
 *   chip_zfec_decode        <- decoding::zfec        src/decoding.rs:34-51
 *   chip_zfec_decode_shares <- decoding::zfec_chunks src/decoding.rs:21-32
 *                              (with explicit share indices; see below)
 *   chip_bao_decode         <- decoding::bao         src/decoding.rs:53-60
 *
 * plus the glue that calls them:
 *   chip_encode             <- encoding::encode      src/encoding.rs:86-172
 *   chip_decode             <- decoding::decode      src/decoding.rs:80-114
 * the host stages that bracket the GPU path (run on host threads):
 *   chip_snap_compress      <- encoding::snap        src/encoding.rs:16-28
 *   chip_snap_decompress    <- decoding::snap        src/decoding.rs:70-77
 *   chip_ecies_encrypt      <- encoding::ecies       src/encoding.rs:30-36
 *   chip_ecies_decrypt      <- decoding::ecies       src/decoding.rs:62-68
 * the streaming hasher:
 *   chip_bao_hasher_*       <- utils::BaoHasher      src/utils.rs:104-137
 * and helpers:
 *   chip_calc_padding_len   <- utils::calc_padding_len src/utils.rs:47-58
 *
 * Conventions
 *   - Plain pointers and sizes, no torch/HIP types in signatures.  Streams are
 *     passed as `void*` (a hipStream_t; NULL = the library's per-thread stream).
 *   - Output buffers are caller-allocated (the Rust shim does
 *     Vec::with_capacity + set_len).  Sizes are computable up front with the
 *     *_len helpers.  A too-small buffer returns CHIP_ERR_BUFFER_TOO_SMALL.
 *   - Every entry point that fills a caller buffer and succeeds writes EVERY
 *     byte below the length it reports in *out_len (chip_zfec_encode: all
 *     m*chunk_len bytes), never a byte at or past out_cap: a caller may hand
 *     over uninitialised memory (the Rust shim's set_len, the Python
 *     wrappers' uninitialised bytes objects).  tests/test_gpu_written.py
 *     checks it for each such entry point with 0xA5- and 0x5A-filled buffers.
 *   - Every function returns a chip_status (0 = OK).  The mapping to
 *     CarbonadoError (src/error.rs) is given per code.
 *   - Host-pointer entry points are synchronous and thread-safe (one HIP
 *     stream + grow-only device scratch per calling thread).  The *_dev batch
 *     entry points take device pointers, enqueue on the given stream and
 *     return without synchronising.
 *   - There is no CPU fallback: with no usable gfx950 device every compute
 *     entry point returns CHIP_ERR_NO_DEVICE.
 */
#ifndef CARBONADO_HIP_H
#define CARBONADO_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h> /* ssize_t */

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define CHIP_API __attribute__((visibility("default")))
#else
#define CHIP_API
#endif

#define CHIP_ABI_VERSION 5
#define CHIP_HASH_LEN 32   /* bao::HASH_SIZE */
#define CHIP_SLICE_LEN 1024 /* constants.rs:9 SLICE_LEN */
#define CHIP_FEC_K 4        /* constants.rs:11 FEC_K */
#define CHIP_FEC_M 8        /* constants.rs:13 FEC_M */
#define CHIP_HEADER_LEN 160  /* file.rs:257-259 Header::len() */

/* constants.rs:49-56 (bitmask_enum, declaration order) */
#define CHIP_FORMAT_ECIES 1u
#define CHIP_FORMAT_SNAPPY 2u
#define CHIP_FORMAT_BAO 4u
#define CHIP_FORMAT_ZFEC 8u

typedef enum chip_status {
    CHIP_OK = 0,
    CHIP_ERR_INVALID_ARG = 1,        /* null pointer / impossible size          */
    CHIP_ERR_BUFFER_TOO_SMALL = 2,   /* caller buffer shorter than required     */
    CHIP_ERR_UNEVEN_ZFEC_CHUNKS = 3, /* CarbonadoError::UnevenZfecChunks  error.rs:61-63 */
    CHIP_ERR_HASH_DECODE = 4,        /* CarbonadoError::HashDecodeError   error.rs:77-79 */
    CHIP_ERR_BAO_HASH_MISMATCH = 5,  /* CarbonadoError::BaoDecodeError(HashMismatch) error.rs:45-47 */
    CHIP_ERR_BAO_TRUNCATED = 6,      /* CarbonadoError::BaoDecodeError(Truncated)    error.rs:45-47 */
    CHIP_ERR_ZFEC = 7,               /* CarbonadoError::ZfecError          error.rs:49-51 */
    CHIP_ERR_ENCODE_ZFEC_PADDING = 8,/* CarbonadoError::EncodeZfecPaddingError error.rs:85-87 */
    CHIP_ERR_ENCODE_INVALID_CHUNK_LENGTH = 9, /* error.rs:89-91 */
    CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT = 10, /* error.rs:93-95 */
    CHIP_ERR_UNSUPPORTED_FORMAT = 11,/* reserved (ABI 1: Ecies/Snappy bits)       */
    CHIP_ERR_UNNECESSARY_SCRUB = 12, /* CarbonadoError::UnnecessaryScrub       error.rs:65-67 */
    CHIP_ERR_SCRUBBED_PADDING_MISMATCH = 13, /* ScrubbedPaddingMismatch         error.rs:69-71 */
    CHIP_ERR_SCRUBBED_LENGTH_MISMATCH = 14,  /* ScrubbedLengthMismatch          error.rs:73-75 */
    CHIP_ERR_INVALID_SCRUBBED_HASH = 15,     /* InvalidScrubbedHash             error.rs:81-83 */
    CHIP_ERR_SNAP = 16,              /* snappy framing error: StdIoError / SnapError error.rs:7,35 */
    CHIP_ERR_ECIES = 17,             /* CarbonadoError::EciesError (bad key, bad tag) error.rs:43 */
    CHIP_ERR_SECP256K1 = 18,         /* secp256k1::Error (bad key / message / signature), error.rs:55 */
    CHIP_ERR_INVALID_HEADER_LENGTH = 19, /* CarbonadoError::InvalidHeaderLength  error.rs:113-115 */
    CHIP_ERR_INVALID_MAGIC = 20,     /* CarbonadoError::InvalidMagicNumber    error.rs:97-99 */
    CHIP_ERR_NO_DEVICE = 100,        /* new variant: no usable gfx950 device     */
    CHIP_ERR_DEVICE = 101            /* new variant: HIP runtime error            */
} chip_status;

/* structs.rs:12-44 EncodeInfo, field for field (u32 / f32 / u16) */
typedef struct chip_encode_info {
    uint32_t input_len;
    uint32_t output_len;
    uint32_t bytes_compressed;
    float compression_factor;
    uint32_t bytes_encrypted;
    uint32_t bytes_ecc;
    uint32_t bytes_verifiable;
    float amplification_factor;
    uint32_t padding_len;
    uint32_t chunk_len;
    uint16_t verifiable_slice_count;
    uint16_t chunk_slice_count;
} chip_encode_info;

/* The two values ecies::encrypt draws from thread_rng (ephemeral secret key,
 * AES-GCM nonce).  NULL fields (or a NULL struct) = fresh random values, as the
 * reference; injected values make encode() deterministic for parity tests.
 * For batch calls the arrays hold one value per object. */
typedef struct chip_ecies_inject {
    const uint8_t *ephemeral_sk; /* 32 bytes per object, 0 < k < n */
    const uint8_t *nonce;        /* 16 bytes per object */
} chip_ecies_inject;

/* ---- library ---------------------------------------------------------- */
CHIP_API int chip_abi_version(void);
CHIP_API const char *chip_strerror(int status);
/* Initialise the HIP context on `device` (idempotent).  CHIP_ERR_NO_DEVICE if
 * no gfx950 device is visible. */
CHIP_API int chip_init(int device);
/* Last HIP error string seen by this thread (for CHIP_ERR_DEVICE). */
CHIP_API const char *chip_last_device_error(void);

/* ---- flat-file container (file.rs) -------------------------------------- */
/* file.rs:24-43 Header, deserialized.  `has_metadata` = Option::Some (the
 * reference reads eight zero bytes as None, file.rs:379-384). */
typedef struct chip_header {
    uint8_t pubkey[33];     /* compressed secp256k1 point */
    uint8_t hash[32];       /* bao hash */
    uint8_t signature[64];  /* BIP-340 Schnorr signature over `hash` */
    uint8_t format;
    uint8_t chunk_index;
    uint32_t encoded_len;
    uint32_t padding_len;
    uint8_t metadata[8];
    uint8_t has_metadata;
} chip_header;
/* BIP-340 over secp256k1 (secp256k1 0.28 Keypair::sign_schnorr, used by
 * Header::new file.rs:269-271).  aux = 32 bytes of auxiliary randomness, or
 * NULL for fresh random bytes (the reference draws them from thread_rng). */
CHIP_API int chip_schnorr_sign(const uint8_t *sk, uint64_t sk_len, const uint8_t *msg32, const uint8_t *aux32,
                               uint8_t *sig64);
/* pubkey: 32-byte x-only, 33-byte compressed or 65-byte uncompressed. */
CHIP_API int chip_schnorr_verify(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *msg32,
                                 const uint8_t *sig64);
/* Header::new (file.rs:263-289): signs `hash` with `sk`, stores `pk` (33 or
 * 65 bytes; kept compressed).  metadata: 8 bytes or NULL (None). */
CHIP_API int chip_header_new(const uint8_t *sk, uint64_t sk_len, const uint8_t *pk, uint64_t pk_len,
                             const uint8_t *hash, uint64_t hash_len, uint8_t format, uint8_t chunk_index,
                             uint32_t encoded_len, uint32_t padding_len, const uint8_t *metadata8,
                             const uint8_t *aux32, chip_header *out);
/* Header::try_to_vec (file.rs:292-335): CHIP_HEADER_LEN bytes. */
CHIP_API int chip_header_to_bytes(const chip_header *h, uint8_t *out160);
/* Header::try_from(&[u8]) (file.rs:116-154): magic, pubkey, signature check.
 * A slice shorter than the parsed 159 bytes is CHIP_ERR_INVALID_HEADER_LENGTH
 * (the reference panics, file.rs:126). */
CHIP_API int chip_header_parse(const uint8_t *bytes, uint64_t len, chip_header *out);
/* file::encode (file.rs:409-440): header || encode(pubkey, input, level);
 * pk NULL/0 = derived from sk.  Randomness: `inject` (ECIES) and `aux32`
 * (signature) or NULL for fresh values.  Needs CHIP_HEADER_LEN +
 * chip_encode_max_len(n) bytes (a short buffer reports that in *out_len). */
CHIP_API int chip_file_encode(const uint8_t *sk, uint64_t sk_len, const uint8_t *pk, uint64_t pk_len,
                              const uint8_t *in, uint64_t n, uint8_t level, const uint8_t *metadata8,
                              const chip_ecies_inject *inject, const uint8_t *aux32, uint8_t *out, uint64_t out_cap,
                              uint64_t *out_len, chip_encode_info *info);
/* file::decode (file.rs:395-407): parse + verify the header, then decode(). */
CHIP_API int chip_file_decode(const uint8_t *sk, uint64_t sk_len, const uint8_t *in, uint64_t n, chip_header *hdr,
                              uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* ---- batch buffers ------------------------------------------------------ */
/* Device memory for batch buffers.  From 1 GiB up it is class-balanced:
 * built from 8 MiB physical pieces chosen across the HBM's write "classes"
 * (timed at allocation) and mapped in a shuffled order behind one fresh
 * virtual range, so streaming writes spread over every class (DESIGN.md §2,
 * §3 K1: 4-of-8 encode at 0.77-0.78 of the roofline vs 0.63-0.67 over one
 * hipMalloc).  Smaller buffers (or CHIP_ALLOC=contiguous): physically
 * contiguous memory where free, else hipMalloc.  Any 16-B aligned device
 * memory works with the batch entry points; this is where they run fastest. */
CHIP_API int chip_device_alloc(uint64_t bytes, void **ptr);
CHIP_API int chip_device_free(void *ptr);
/* For a class-balanced buffer from chip_device_alloc: how many memory
 * classes the allocation found and used, and the seconds it took.
 * CHIP_ERR_INVALID_ARG for any other pointer. */
CHIP_API int chip_device_alloc_info(const void *ptr, uint32_t *classes_found, uint32_t *classes_used,
                                    double *seconds);
/* The same, with the signatures torch.cuda.memory.CUDAPluggableAllocator
 * loads (size, device, stream): a torch MemPool over these hands out
 * contiguous tensors (carbonado_amd.device.empty_batch). */
CHIP_API void *chip_torch_alloc(ssize_t size, int device, void *stream);
CHIP_API void chip_torch_free(void *ptr, ssize_t size, int device, void *stream);

/* Diagnostic: the device address of the run-queue counter block the batch
 * kernels use on `stream` (NULL = the calling thread's own stream), assigning
 * one if the stream has none yet.  Every live stream has a block of its own
 * (DESIGN.md §3 K1 "Counter blocks"). */
CHIP_API int chip_stream_queue_block(void *stream, uint64_t *addr);

/* Diagnostic: where this process's host-copy path sits on the box, as a JSON
 * object: the GPU's PCI address and NUMA node, the calling thread's pinned
 * staging ring's node, the copy workers and the nodes of the CPUs they last
 * copied on.  The ring and the workers are placed on the GPU's node
 * (CHIP_NUMA=0: runtime defaults).  *len = bytes needed including the NUL;
 * a short buffer returns CHIP_ERR_BUFFER_TOO_SMALL. */
CHIP_API int chip_host_topology(char *json, uint64_t cap, uint64_t *len);

/* ---- size helpers (host only, no device needed) ----------------------- */
/* utils.rs:47-58 with FEC_K generalised to k: target = ceil(n/(1024k))*1024k,
 * padding = target - n, chunk_len = target / k (integer maths; the reference's
 * f64 is exact for every length it can hold). */
CHIP_API int chip_calc_padding_len(uint64_t input_len, uint32_t k, uint32_t *padding, uint32_t *chunk_len);
/* m * chunk_len */
CHIP_API uint64_t chip_zfec_encoded_len(uint64_t input_len, uint32_t k, uint32_t m);
/* 8 + n + 64 * (max(1, ceil(n/1024)) - 1) */
CHIP_API uint64_t chip_bao_encoded_len(uint64_t content_len);
/* upper bound of chip_encode's output for an n-byte input (any format bits) */
CHIP_API uint64_t chip_encode_max_len(uint64_t input_len);
/* upper bound of chip_snap_compress's output */
CHIP_API uint64_t chip_snap_max_len(uint64_t input_len);

/* ---- stage functions (host buffers) ----------------------------------- */
/* encoding::zfec (encoding.rs:48-81).  out receives m*chunk_len bytes laid out
 * shard-major [S0|S1|...|S(m-1)]; S0..S(k-1) are the zero-padded input.
 * The reference fixes (k, m) = (FEC_K, FEC_M) = (4, 8); other values expose
 * the kernel layer (1 <= k <= m <= 256). */
CHIP_API int chip_zfec_encode(uint32_t k, uint32_t m, const uint8_t *in, uint64_t n, uint8_t *out,
                     uint64_t out_cap, uint32_t *padding, uint32_t *chunk_len);

/* decoding::zfec (decoding.rs:34-51): len % m != 0 -> CHIP_ERR_UNEVEN_ZFEC_CHUNKS;
 * shards are indexed by position 0..m as the reference does (decoding.rs:24-25).
 * out receives k*(len/m) - padding bytes. */
CHIP_API int chip_zfec_decode(uint32_t k, uint32_t m, const uint8_t *in, uint64_t len, uint32_t padding,
                     uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* decoding::zfec_chunks (decoding.rs:21-32) with EXPLICIT share indices:
 * shares[s] holds chunk_len bytes of share idx[s].  The reference numbers the
 * surviving shares by position, which mislabels them once a data shard is
 * lost; this entry point takes the true
 * indices.  Primary shares are used where present, secondaries fill the gaps
 * in the order given.  Fewer than k distinct shares -> CHIP_ERR_ZFEC. */
CHIP_API int chip_zfec_decode_shares(uint32_t k, uint32_t m, const uint8_t *const *shares,
                            const uint32_t *idx, uint32_t nshares, uint64_t chunk_len,
                            uint32_t padding, uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* encoding::bao (encoding.rs:38-44 -> bao::encode::encode): combined pre-order
 * encoding (u64 LE length, 64-byte parents, 1 KiB chunks) and the root hash
 * (== BLAKE3(in)). */
CHIP_API int chip_bao_encode(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                    uint64_t *out_len, uint8_t hash[CHIP_HASH_LEN]);

/* decoding::bao (decoding.rs:53-60): hash_len != 32 -> CHIP_ERR_HASH_DECODE
 * (utils.rs:37-45); any node mismatch -> CHIP_ERR_BAO_HASH_MISMATCH; stream
 * shorter than its header implies -> CHIP_ERR_BAO_TRUNCATED. */
CHIP_API int chip_bao_decode(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len,
                    uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* BLAKE3 of a host buffer, computed on the device (bao root hash). */
CHIP_API int chip_blake3(const uint8_t *in, uint64_t n, uint8_t hash[CHIP_HASH_LEN]);

/* ---- host stages (host buffers, host threads; no device) --------------- */
/* encoding::snap (encoding.rs:16-28): snap 1.1 FrameEncoder output (stream
 * identifier, one chunk per 64 KiB block with the masked CRC-32C, raw when
 * compression saves < 1/8).  An empty input gives an empty output. */
CHIP_API int chip_snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                                uint64_t *out_len);
/* decoding::snap (decoding.rs:70-77): FrameDecoder::read_to_end.  Corrupt
 * frames or CRC mismatch -> CHIP_ERR_SNAP.  A short buffer returns
 * CHIP_ERR_BUFFER_TOO_SMALL with *out_len = the decompressed size. */
CHIP_API int chip_snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                                  uint64_t *out_len);
/* encoding::ecies (encoding.rs:30-36 -> ecies 0.2.6 encrypt): receiver key of
 * 33/64/65 bytes; output eph_pub(65) || nonce(16) || tag(16) || ciphertext,
 * n + 97 bytes.  inject = NULL for random ephemeral key and nonce. */
CHIP_API int chip_ecies_encrypt(const uint8_t *pubkey, uint64_t pubkey_len, const chip_ecies_inject *inject,
                                const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                                uint64_t *out_len);
/* decoding::ecies (decoding.rs:62-68 -> ecies::decrypt): bad key, short input
 * or tag mismatch -> CHIP_ERR_ECIES. */
CHIP_API int chip_ecies_decrypt(const uint8_t *secret_key, uint64_t sk_len, const uint8_t *in, uint64_t n,
                                uint8_t *out, uint64_t out_cap, uint64_t *out_len);
/* secp256k1 public key (65 bytes, uncompressed) of a 32-byte secret key. */
CHIP_API int chip_ecies_public_key(const uint8_t *secret_key, uint8_t pubkey[65]);

/* ---- pipeline glue (host buffers) -------------------------------------- */
/* encoding::encode (encoding.rs:86-172): snap -> ecies on the host, then
 * zfec -> bao on the device (the zfec output stays device-resident for the
 * bao stage).  pubkey is used only with the Ecies bit. */
CHIP_API int chip_encode(uint8_t format, const uint8_t *pubkey, uint64_t pubkey_len,
                const chip_ecies_inject *inject, const uint8_t *in, uint64_t n, uint8_t *out,
                uint64_t out_cap, uint64_t *out_len, uint8_t hash[CHIP_HASH_LEN], chip_encode_info *info);
/* decoding::decode (decoding.rs:80-114): bao -> zfec on the device, then
 * ecies -> snap on the host.  With the Snappy bit the output size is only
 * known after decompression: a short buffer returns CHIP_ERR_BUFFER_TOO_SMALL
 * with *out_len = the size needed.  After any other error out's bytes are
 * unspecified: never content that failed verification (the host stages may
 * run on the content while the device verifies it; a failed verdict wipes
 * what they wrote). */
CHIP_API int chip_decode(const uint8_t *secret_key, uint64_t sk_len, const uint8_t *hash, uint64_t hash_len,
                const uint8_t *in, uint64_t n, uint32_t padding, uint8_t format, uint8_t *out,
                uint64_t out_cap, uint64_t *out_len);

/* ---- device-resident batch API (the throughput path) ------------------ */
/* `count` objects of `n` bytes each; object o's input at d_in + o*in_stride
 * (bytes beyond n inside the padded object read as zero, exactly as
 * encoding.rs:53-55 pads), its m*chunk_len-byte output at d_out + o*out_stride.
 * d_in, d_out, in_stride and out_stride must be multiples of 16
 * (CHIP_ERR_INVALID_ARG otherwise); multiples of 256 are the fast layout (every
 * row's shards then start on a 128-B memory line: at a 16-B pitch each piece
 * a wave loads straddles two lines and the kernels fetch 1.21x the input,
 * DESIGN.md §2).  Every batch entry point below refuses
 * (CHIP_ERR_INVALID_ARG) strides under the row length when count > 1: rows
 * would overlap.
 * In place: d_out == d_in (and out_stride == in_stride) means each object's
 * first n bytes already are its data shards; only the m-k parity shards are
 * written and the padding bytes [n, k*chunk_len) are zeroed (SURVEY.md 8d
 * "aliased": 32 MiB of traffic per 16 MiB object instead of 48). */
CHIP_API int chip_zfec_encode_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                               uint64_t n, uint64_t count, uint8_t *d_out, uint64_t out_stride,
                               void *stream);
/* Diagnostic (ABI 5): the memory pattern of chip_zfec_encode_batch_dev with
 * the same arguments — the same loads, stores, grid, run queue and LDS
 * footprint — with the GF(2^8) arithmetic taken out (computed row q is the
 * XOR of the k data shards with every byte XOR q, NOT parity).  Its rate is what this box's HBM
 * gives the encode's access pattern on these buffers: the ceiling the encode
 * is compared with (bench.py box_ceiling).  (k, m) = (4, 8) or (8, 16);
 * d_out != d_in; CHIP_ERR_ZFEC for other shapes. */
CHIP_API int chip_hbm_pattern_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                                        uint64_t n, uint64_t count, uint8_t *d_out, uint64_t out_stride,
                                        void *stream);
/* Erasure decode of `count` encoded objects (chunk_len-byte shards, shard i of
 * object o at d_in + o*in_stride + i*chunk_len).  idx[0..nshares) names the
 * shares that survive (same pattern for every object); the k*chunk_len data
 * bytes of object o go to d_out + o*out_stride (caller truncates `padding`).
 * Pointers, strides and chunk_len must be multiples of 16. */
CHIP_API int chip_zfec_decode_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                               uint64_t chunk_len, const uint32_t *idx, uint32_t nshares,
                               uint64_t count, uint8_t *d_out, uint64_t out_stride, void *stream);
/* bao encode of `count` objects of n bytes: object o's stream (length
 * chip_bao_encoded_len(n)) at d_out + o*out_stride, its hash at
 * d_hash + 32*o.  d_scratch must hold chip_bao_scratch_len(n, count) bytes. */
CHIP_API uint64_t chip_bao_scratch_len(uint64_t n, uint64_t count);
CHIP_API int chip_bao_encode_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash,
                              void *d_scratch, void *stream);
/* bao verify-decode of `count` streams whose content length is n (checked
 * against each header): content of object o to d_out + o*out_stride; per
 * object status (0 or a chip_status) to d_status[o] (uint32). */
CHIP_API int chip_bao_decode_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                              const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride,
                              uint32_t *d_status, void *d_scratch, void *stream);

/* encode() (encoding.rs:86-172) of `count` DEVICE-resident objects for the
 * formats whose stages all run on the device (Bao and/or Zfec bits only;
 * Snappy/Ecies bits give CHIP_ERR_INVALID_ARG — they are host stages, see
 * chip_encode_host_batch).  Object o: n bytes at d_in + o*in_stride; its
 * encoding (*out_len bytes, the same for every object) at d_out +
 * o*out_stride, its hash at d_hash + 32*o (zeros without Bao,
 * encoding.rs:145), *info = its EncodeInfo (may be NULL).  Zfec|Bao runs
 * fused: one kernel computes the 8 shards, hashes them on chip and writes
 * them straight into their chunk slots of the bao stream (no zfec buffer,
 * the shards cross HBM once; CHIP_FUSED=0 selects the two-kernel path).
 * d_scratch: chip_encode_scratch_len(format, n, count) bytes.  Pointers and
 * strides must be multiples of 16 (CHIP_ERR_INVALID_ARG otherwise), except
 * d_out and out_stride with the Bao bit for streams of more than 512 chunks
 * (objects over 128 KiB at Zfec|Bao, 512 KiB at Bao), which the kernels
 * write at any 8-B phase: there they need only be multiples of 8.  The fast layout for those puts
 * each stream at 56 mod 64 (d_out and out_stride), so that after its 8-byte
 * header every chunk and parent node starts on a 64-B boundary and no store
 * splits a 64-B segment (rows of a 256-B multiple pitch, the stream 56 bytes
 * in).  Enqueued on `stream`, not synchronised.  Replaces, for these levels,
 * encode() = zfec (encoding.rs:121-138) -> bao (encoding.rs:140-147) in one
 * call per batch. */
CHIP_API uint64_t chip_encode_scratch_len(uint8_t format, uint64_t n, uint64_t count);
CHIP_API int chip_encode_batch_dev(uint8_t format, const uint8_t *d_in, uint64_t in_stride, uint64_t n,
                                   uint64_t count, uint8_t *d_out, uint64_t out_stride, uint64_t *out_len,
                                   uint8_t *d_hash, chip_encode_info *info, void *d_scratch, void *stream);

/* decode() (decoding.rs:80-114) of `count` DEVICE-resident encodings of the
 * device-only formats (Bao and/or Zfec bits; Snappy/Ecies bits give
 * CHIP_ERR_INVALID_ARG).  Object o: the in_len-byte encoding at d_in +
 * o*in_stride, its bao hash at d_hash + 32*o (device), all with the zfec
 * `padding` of one chip_encode_batch_dev; decoded bytes (*out_len, the same
 * for every object) at d_out + o*out_stride, status (0 or a chip_status:
 * CHIP_ERR_BAO_HASH_MISMATCH for a corrupted stream or a header that
 * disagrees with in_len) at d_status[o].  At Bao|Zfec every node of the
 * stream is verified and only the primaries' bytes are written (the shards
 * are indexed by position, decoding.rs:95-99: decode = the 4 data shards,
 * padding dropped).  d_scratch: chip_decode_scratch_len(format, in_len,
 * count) bytes.  Pointers and strides multiples of 16, except d_in and
 * in_stride with the Bao bit for streams of more than 512 chunks: multiples
 * of 8, and 56 mod 64 (as chip_encode_batch_dev's fast layout writes them)
 * is the fast layout for reading them too.  Enqueued on `stream`. */
CHIP_API uint64_t chip_decode_scratch_len(uint8_t format, uint64_t in_len, uint64_t count);
CHIP_API int chip_decode_batch_dev(uint8_t format, const uint8_t *d_in, uint64_t in_stride, uint64_t in_len,
                                   uint64_t count, const uint8_t *d_hash, uint32_t padding, uint8_t *d_out,
                                   uint64_t out_stride, uint64_t *out_len, uint32_t *d_status, void *d_scratch,
                                   void *stream);

/* ---- slices and scrub (decoding.rs:116-212) ----------------------------- */
/* Chunk range of a bao slice request [start, start+len) over n content bytes,
 * bao's rules: at least one chunk; a start at/after the end selects the last
 * chunk.  Byte length of the extracted slice (header + parents + chunks). */
CHIP_API uint64_t chip_bao_slice_len(uint64_t content_len, uint64_t start, uint64_t len);
/* extract_slice (decoding.rs:116-127) with a u64 slice index (the reference
 * computes `index * SLICE_LEN` in u16, which wraps for index >= 64): the bao
 * slice for content bytes [index*1024, index*1024 + slice_len) of the
 * combined encoding `enc`.  Pure byte selection along the tree. */
CHIP_API int chip_bao_extract_slice(const uint8_t *enc, uint64_t len, uint64_t index, uint64_t slice_len,
                                    uint8_t *out, uint64_t out_cap, uint64_t *out_len);
/* verify_slice (decoding.rs:129-149): verify the `count` 1 KiB slices starting
 * at slice `index` of the combined encoding against `hash` (every chunk in the
 * range and every parent above it, re-hashed on the device) and return their
 * content.  Corruption outside the range does not fail the slice. */
CHIP_API int chip_bao_verify_slice(const uint8_t *hash, uint64_t hash_len, const uint8_t *enc, uint64_t len,
                                   uint64_t index, uint64_t count, uint8_t *out, uint64_t out_cap,
                                   uint64_t *out_len);
/* scrub (decoding.rs:151-212) for a level-12/14/15 stream: if the stream
 * verifies -> CHIP_ERR_UNNECESSARY_SCRUB; else verify each of the 8 shards'
 * slices, zfec-decode from the good shards with their TRUE share indices
 * (the reference numbers survivors by position, decoding.rs:187 -> :24-25),
 * re-encode zfec + bao and return the stream if its length and hash match.
 * out must hold `len` bytes. */
CHIP_API int chip_scrub(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len,
                        uint32_t padding, uint32_t chunk_len, uint8_t *out, uint64_t out_cap, uint64_t *out_len);
/* scrub (decoding.rs:151-212) of `count` DEVICE-resident Bao|Zfec streams of
 * `len` bytes each (stream o at d_in + o*in_stride, its expected hash at
 * d_hash + 32*o, device), all with one EncodeInfo (padding, chunk_len; the
 * content is 8*chunk_len bytes, else CHIP_ERR_ZFEC for the call).  Every
 * node of every stream is verified on the device in one pass, then each
 * stream's shards (the slices decoding.rs:173-183 verifies): status[o]
 * (host) = CHIP_ERR_UNNECESSARY_SCRUB for an intact stream, CHIP_ERR_ZFEC
 * with fewer than 4 authentic shards, else the stream is repaired and
 * status[o] = CHIP_OK or the reference's scrub error (padding / length
 * mismatch, invalid scrubbed hash).  Row o of d_out (d_out + o*out_stride)
 * is written only when status[o] == CHIP_OK (the repaired stream's hash
 * matched); every other row is left untouched.  d_scratch:
 * chip_scrub_scratch_len(len, count) bytes.  Pointers and strides multiples
 * of 8 (the streams at 56 mod 64 are the fast layout, as for
 * chip_encode_batch_dev).  Synchronous: returns when every status is final. */
CHIP_API uint64_t chip_scrub_scratch_len(uint64_t len, uint64_t count);
CHIP_API int chip_scrub_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t len, uint64_t count,
                                  const uint8_t *d_hash, uint32_t padding, uint32_t chunk_len, uint8_t *d_out,
                                  uint64_t out_stride, int32_t *status, void *d_scratch, void *stream);

/* ---- streaming bao hasher (utils.rs:104-137 BaoHasher) ------------------ */
/* A thread-safe append-only hasher (one mutex per hasher, as the reference's
 * RwLock).  update() appends to a growing HBM buffer (the caller's bytes are
 * copied before it returns); finalize() runs the bao kernels over everything
 * appended and returns the root hash (== BLAKE3 of the content); read_all()
 * returns the combined bao encoding (== bao::encode::encode of the content).
 * update() after finalize() -> CHIP_ERR_INVALID_ARG (the reference's encoder
 * panics); finalize() again returns the same hash; read_all() before
 * finalize() -> CHIP_ERR_INVALID_ARG. */
typedef struct chip_bao_hasher chip_bao_hasher;
CHIP_API int chip_bao_hasher_new(chip_bao_hasher **out);
CHIP_API int chip_bao_hasher_update(chip_bao_hasher *h, const uint8_t *buf, uint64_t n);
CHIP_API int chip_bao_hasher_finalize(chip_bao_hasher *h, uint8_t hash[CHIP_HASH_LEN]);
CHIP_API uint64_t chip_bao_hasher_len(chip_bao_hasher *h);
CHIP_API int chip_bao_hasher_read_all(chip_bao_hasher *h, uint8_t *out, uint64_t out_cap, uint64_t *out_len);
CHIP_API void chip_bao_hasher_free(chip_bao_hasher *h);
/* Freed hashers are parked for reuse by the next chip_bao_hasher_new (their
 * streams, and their device buffers while all parked buffers together stay
 * within CHIP_HASHER_PARK_MIB, 3 GiB by default; at most 4 hashers).
 * drop_cache destroys every parked hasher and returns the device bytes it
 * freed; cached_bytes reports what the parked hashers hold (ABI 5). */
CHIP_API uint64_t chip_bao_hasher_drop_cache(void);
CHIP_API uint64_t chip_bao_hasher_cached_bytes(void);

/* ---- host-memory batch (end-to-end: host -> HBM -> host) -------------- */
/* encode() for `count` objects of n bytes that live in HOST memory (object o
 * at in + o*in_stride) into host memory (stream o at out + o*out_stride,
 * length out_len[o]; hash o at hashes + 32*o; EncodeInfo o at info[o], info
 * may be NULL).  Objects are processed in slices over `nslots` device slots,
 * each with its own stream, so the H2D copy of one slice, the kernels of the
 * next and the D2H copy of a third overlap (PCIe full duplex); the host
 * stages (Snappy/Ecies bits) of a slice run on `host_threads` host threads
 * (0 = one per hardware thread, at most 64) while earlier slices are on the
 * device.  out_stride must hold chip_encode_max_len(n).  Pinned host buffers
 * reach the full PCIe rate; pageable ones are staged by the runtime. */
CHIP_API int chip_encode_host_batch(uint8_t format, const uint8_t *pubkey, uint64_t pubkey_len,
                                    const chip_ecies_inject *inject, const uint8_t *in, uint64_t n,
                                    uint64_t count, uint64_t in_stride, uint8_t *out, uint64_t out_stride,
                                    uint64_t *out_len, uint8_t *hashes, chip_encode_info *info,
                                    uint32_t nslots, uint64_t slice_bytes, uint32_t host_threads);

/* decode() for `count` encoded objects in HOST memory (object o: in_len[o]
 * bytes at in + o*in_stride, bao hash at hashes + 32*o, zfec padding[o]) into
 * host memory (out + o*out_stride, out_len[o] bytes).  Device part per slice:
 * H2D, bao verify-decode, zfec (positional shards: the primaries' bytes,
 * decoding.rs:95-99), D2H; the Ecies/Snappy host stages of a slice run on
 * `host_threads` threads while the next slice is on the device.  Per-object
 * results go to status[o] (a chip_status; a short out_stride gives
 * CHIP_ERR_BUFFER_TOO_SMALL with out_len[o] = the size needed); the call
 * returns CHIP_OK when every object decoded, else the first failing status. */
CHIP_API int chip_decode_host_batch(uint8_t format, const uint8_t *secret_key, uint64_t sk_len,
                                    const uint8_t *hashes, const uint8_t *in, const uint64_t *in_len,
                                    uint64_t count, uint64_t in_stride, const uint32_t *padding, uint8_t *out,
                                    uint64_t out_stride, uint64_t *out_len, int32_t *status, uint32_t nslots,
                                    uint64_t slice_bytes, uint32_t host_threads);

#ifdef __cplusplus
}
#endif
#endif /* CARBONADO_HIP_H */
