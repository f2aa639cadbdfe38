/*
 * carbonado_oracle.h — CPU ORACLE for the carbonado zfec/bao hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker (or the timed CPU baseline), never as the
 * thing that produces shipped bytes.  The product path is
 * carbonado_amd/lib/libcarbonado_hip.so (HIP kernels for gfx950).
 *
 * What it restates (plain C, scalar, single thread):
 *   - reference glue: /root/reference/src/encoding.rs:38-81 (bao/zfec stages),
 *     :86-172 (encode() + EncodeInfo), src/decoding.rs:21-60 (zfec/bao
 *     decode stages), :80-114 (decode()), src/utils.rs:37-58 (hash parse,
 *     calc_padding_len), src/constants.rs:8-12,49-56 (K, M, SLICE_LEN, Format).
 *   - third-party arithmetic that is NOT vendored in /root/reference:
 *       zfec-rs 0.1.0 (Cargo.toml:36)  -> Rizzo/zfec fec.c construction:
 *           GF(2^8) with polynomial 0x11D, generator 2; enc_matrix = systematic
 *           form of the Vandermonde matrix at points {0, a^0, a^1, ...}.
 *       bao 0.12.1 -> blake3 1.x (Cargo.toml:13) -> BLAKE3 spec (chunk CVs,
 *           parents, ROOT flag) and the bao combined pre-order encoding.
 *
 * Parity status: the restatement is pinned by published BLAKE3 known-answer
 * vectors (tests/golden/blake3_kat.json) and by self-consistency invariants
 * for zfec (systematic identity, MDS over all k-subsets); zfec-rs itself is
 * absent from this container, so zfec parity bytes are "parity unpinned"
 * against the real crate.
 */
#ifndef CARBONADO_ORACLE_H
#define CARBONADO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/carbonado_hip.h */
enum {
    ORC_OK = 0,
    ORC_ERR_INVALID_ARG = 1,
    ORC_ERR_BUFFER_TOO_SMALL = 2,
    ORC_ERR_UNEVEN_ZFEC_CHUNKS = 3,
    ORC_ERR_HASH_DECODE = 4,
    ORC_ERR_BAO_HASH_MISMATCH = 5,
    ORC_ERR_BAO_TRUNCATED = 6,
    ORC_ERR_ZFEC = 7,
    ORC_ERR_INVALID_VERIFIABLE_SLICE_COUNT = 10,
    ORC_ERR_UNSUPPORTED_FORMAT = 11,
    ORC_ERR_SNAP = 16,
    ORC_ERR_ECIES = 17,
};

/* GF(2^8) */
uint8_t orc_gf_mul(uint8_t a, uint8_t b);
uint8_t orc_gf_inv(uint8_t a);
/* m x k systematic encoding matrix (row-major). 1 <= k <= m <= 256 */
int orc_fec_enc_matrix(unsigned k, unsigned m, uint8_t *mat);
/* invert a k x k matrix in place; returns 0 on success, -1 if singular */
int orc_gf_invert(uint8_t *mat, unsigned k);

/* utils.rs:50-58 generalised to k: pad to a multiple of 1024*k */
void orc_calc_padding_len(uint64_t input_len, unsigned k, uint32_t *padding, uint32_t *chunk_len);

/* encoding::zfec (encoding.rs:48-81) with (k, m) instead of (FEC_K, FEC_M).
 * out must hold m*chunk_len bytes. */
int orc_zfec_encode(unsigned k, unsigned m, const uint8_t *in, uint64_t n,
                    uint8_t *out, uint64_t out_cap, uint32_t *padding, uint32_t *chunk_len);

/* zfec_chunks (decoding.rs:21-32) with explicit share indices.
 * shares[s] points at chunk_len bytes of share idx[s].  Primary shares are
 * preferred, then secondary shares in the order given.  out receives
 * k*chunk_len - padding bytes (out_cap >= that). */
int orc_zfec_decode_shares(unsigned k, unsigned m, const uint8_t *const *shares,
                           const uint32_t *idx, unsigned nshares, uint64_t chunk_len,
                           uint32_t padding, uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* decoding::zfec (decoding.rs:35-51): m contiguous shards, indexed by position */
int orc_zfec_decode(unsigned k, unsigned m, const uint8_t *in, uint64_t len, uint32_t padding,
                    uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* BLAKE3 */
void orc_blake3(const uint8_t *in, uint64_t n, uint8_t out[32]);
void orc_blake3_chunk_cv(const uint8_t *chunk, uint32_t len, uint64_t counter, int is_root,
                         uint32_t cv[8]);
void orc_blake3_parent_cv(const uint32_t left[8], const uint32_t right[8], int is_root,
                          uint32_t cv[8]);

/* bao combined encoding (encoding.rs:38-44 -> bao::encode::encode) */
uint64_t orc_bao_encoded_len(uint64_t n);
int orc_bao_encode(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint8_t hash[32]);
/* decoding::bao (decoding.rs:54-60 -> bao::decode::decode) */
int orc_bao_decode(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len,
                   uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* EncodeInfo (structs.rs:12-44) */
typedef struct {
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
} orc_encode_info;

/* encode() (encoding.rs:86-172) restricted to Format bits Bao (4) | Zfec (8). */
uint64_t orc_encode_max_len(uint64_t n);
int orc_encode(uint8_t format, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
               uint64_t *out_len, uint8_t hash[32], orc_encode_info *info);
/* decode() (decoding.rs:80-114) restricted to Format bits Bao | Zfec. */
int orc_decode(const uint8_t *hash, uint64_t hash_len, const uint8_t *in, uint64_t n,
               uint32_t padding, uint8_t format, uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* deterministic test-input generator shared with the HIP side:
 * key = seed ^ (obj * 0xD1B54A32D192ED03); word w = mix64(key + (w+1) * 0x9E3779B97F4A7C15)
 * (mix64 = SplitMix64 finaliser); byte i = byte (i & 7) of word (i >> 3), little-endian. */
void orc_fill_object(uint64_t seed, uint64_t obj, uint8_t *out, uint64_t n);

/* host_oracle.c: host stages (snappy framing, ECIES) and the full pipeline */
uint32_t orc_crc32c(const uint8_t *p, uint64_t n);
uint64_t orc_snap_max_len(uint64_t n);
int orc_snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
int orc_snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
void orc_sha256(const uint8_t *in, uint64_t n, uint8_t out[32]);
void orc_hmac_sha256(const uint8_t *key, uint64_t kl, const uint8_t *msg, uint64_t n, uint8_t out[32]);
int orc_ecies_public_key(const uint8_t sk[32], uint8_t out[65]);
int orc_ecies_encrypt(const uint8_t *pub, uint64_t pklen, const uint8_t eph_sk[32], const uint8_t nonce[16],
                      const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
int orc_ecies_decrypt(const uint8_t sk[32], const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                      uint64_t *out_len);
int orc_encode_full(uint8_t format, const uint8_t *pub, uint64_t pklen, const uint8_t eph_sk[32],
                    const uint8_t nonce[16], const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                    uint64_t *out_len, uint8_t hash[32], orc_encode_info *info);

#ifdef __cplusplus
}
#endif
#endif
