// host_stages.hpp — the host-side stages that bracket the GPU path in
// encode()/decode() (encoding.rs:16-36, decoding.rs:62-77): snappy framing and
// ECIES.  They run on host threads, overlapped with the device pipeline by
// chip_encode_host_batch; the GPU path itself starts at zfec.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>

namespace chip {
namespace host {

// CRC-32C (Castagnoli), as used by the snappy framing format.
uint32_t crc32c(const uint8_t *p, size_t n);

// ---- snappy (snap 1.1.0: write::FrameEncoder / read::FrameDecoder) -------
// Upper bound of snap_compress's output for n input bytes.
uint64_t snap_max_len(uint64_t n);
// Framed stream of `in` into out[0..cap).  0 = ok, else a CHIP status.
int snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
// Decompressed size of a framed stream (validates chunk structure, not CRCs).
int snap_decompressed_len(const uint8_t *in, uint64_t n, uint64_t *len);
// Full decode with CRC checks.
int snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);

// ---- ECIES (ecies 0.2.6 defaults: secp256k1, uncompressed keys, HKDF-SHA256,
// AES-256-GCM with a 16-byte nonce) ----------------------------------------
constexpr uint64_t ECIES_OVERHEAD = 65 + 16 + 16;
// eph_sk / nonce: injected ephemeral secret (32 B) and nonce (16 B), or null
// for fresh random values (the reference draws both from thread_rng).
int ecies_encrypt(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                  const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
// pre_key / pre_eph (optional): a key already derived (ecies_derive_key) for
// the ephemeral public key pre_eph, used when the envelope's own equals it.
int ecies_decrypt(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                  uint64_t cap, uint64_t *out_len, const uint8_t *pre_key = nullptr, const uint8_t *pre_eph = nullptr);
// ecies_decrypt then snap_decompress (decoding.rs:101-111) in one pass over
// the ciphertext: same output and status codes, no full-size plaintext buffer.
// `window`: DECRYPT_SNAP_WINDOW bytes of caller scratch reused across calls
// (null: a per-thread buffer).  On a bad tag every byte written to `out` and
// the window are wiped.
constexpr uint64_t DECRYPT_SNAP_WINDOW = 256u << 10;
int ecies_decrypt_snap(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                       uint64_t cap, uint64_t *out_len, uint8_t *window = nullptr, const uint8_t *pre_key = nullptr,
                       const uint8_t *pre_eph = nullptr);
// Public key (65 B uncompressed) of a 32-byte secret; for tests and tooling.
int ecies_public_key(const uint8_t *secret, uint8_t out[65]);

// The key material of one ecies_encrypt, split from the bytes: the ephemeral
// public key (the envelope's first 65 bytes) and the AES-256-GCM key.  Its
// cost is two scalar multiplications, independent of the data, so a batch
// computes it ahead (encode() from host memory: while the slice's slot is
// still busy on the device).  ecies_peer parses and checks the receiver key
// once per batch (65 B uncompressed out); ecies_prepare draws (eph_sk null)
// or takes the ephemeral secret.  A prepared key is used once, then wiped.
struct EciesKey {
    uint8_t eph_pub[65];
    uint8_t key[32];
};
int ecies_peer(const uint8_t *pubkey, uint64_t pubkey_len, uint8_t peer[65]);
int ecies_prepare(const uint8_t peer[65], const uint8_t *eph_sk, EciesKey *out);
// The same with its two scalar multiplications (k·G, k·P) handed to run2,
// which calls f(0) and f(1), side by side or not, and returns once both are
// done (a caller that holds the stage pool runs them on its workers).
int ecies_prepare_with(const uint8_t peer[65], const uint8_t *eph_sk, EciesKey *out,
                       const std::function<void(const std::function<void(int)> &)> &run2);
void ecies_key_wipe(EciesKey *k);

// memcpy into pinned staging memory that only the DMA engine reads next:
// non-temporal (streaming) stores skip the read-for-ownership of every
// destination line and keep it out of the CPU caches (AVX2; memcpy without
// it, or with CHIP_NT_COPY=0).
void ring_copy(void *dst, const void *src, size_t n);
// The host-made part of a Zfec|Bao stream (encode() from host memory): its
// header (u64 LE zl) and data chunk i = src[1024 i, 1024 i + 1024), zero past
// n, at out + coff[i] for i < nd (the data shards of the zfec output are the
// zero-padded input itself).  Streaming stores for the whole lines.
void fill_data_chunks(uint8_t *out, const uint64_t *coff, uint64_t nd, uint64_t zl, const uint8_t *src, uint64_t n);
// chunks [c0, c1) only (no header)
void fill_chunk_range(uint8_t *out, const uint64_t *coff, uint64_t c0, uint64_t c1, const uint8_t *src, uint64_t n);

// Where the chunks of the stream being made go: out + coff[i], i < nd.
// complete: every chunk the output touches is written (with the stream's
// header: content length zl), so no contiguous output is needed; the zero
// chunks after them are the caller's.
struct ChunkSink {
    uint8_t *out;
    const uint64_t *coff;
    uint64_t nd;
    bool complete = false;
    uint64_t zl = 0;
};
// ECIES over snap_compress(in) (snap) or over in, in one pass: each 64 KiB
// block is framed into `window` (SNAP_ECIES_WINDOW bytes of caller scratch)
// and encrypted into out.  With a sink (encode() from host memory at
// Ecies|Zfec|Bao) the block's ciphertext goes to the second half of the
// window first and is cut from there into the stream's chunks at their slots
// (and streamed into out, if given: non-temporal, out being pinned staging
// only the DMA reads; CHIP_NT_STAGE=0 plain stores).  Without `complete`,
// chunks [1, *filled) are placed and the caller places the rest once it knows
// the stream's geometry matches the sink's; with it, out may be null, the
// header and chunks [0, *filled) are placed (the last one zero padded) and the
// caller zeroes [*filled, nd) once the geometry is confirmed.  Output
// identical to snap_compress + ecies_encrypt.
constexpr uint64_t SNAP_ECIES_WINDOW = 2 * (64 + 65536 + 65536 / 6);
// prepared: the key material from ecies_prepare (pubkey / eph_sk unused then).
int ecies_encrypt_stream(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                         const uint8_t *in, uint64_t n, bool snap, uint8_t *out, uint64_t cap, uint64_t *out_len,
                         uint8_t *window, const ChunkSink *sink, uint64_t *filled,
                         const EciesKey *prepared = nullptr);
// snap_compress with the same sink (encode() at Snappy|Zfec|Bao): the frame's
// chunks [0, *filled) placed as they complete, `out` optional when complete.
int snap_compress_stream(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                         uint8_t *window, const ChunkSink *sink, uint64_t *filled);
// ecies_encrypt_stream(.., snap = true, no sink) for one object of at least
// STAGE_PAR_MIN bytes on a few threads (encode()'s single-object path): the
// snappy blocks compressed on persistent workers and the caller
// (CHIP_STAGE_THREADS, default 8 with the caller; 1 = this thread only), the
// key agreement on one worker meanwhile; then AES-GCM over 16-B aligned
// pieces of the frame, one per thread, the GHASH parts joined (gcm_vaes.hpp).
// Same bytes; a smaller object, a CPU without the VAES path, or a pool busy
// with another call takes the one-thread path.
constexpr uint64_t STAGE_PAR_MIN = 256 * 1024;
int ecies_encrypt_par(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                      const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                      uint8_t *window);
// ecies_decrypt_snap for one object of at least STAGE_PAR_MIN bytes of
// ciphertext on the same pool: AES-GCM over 16-B aligned pieces into a
// plaintext buffer, the tag checked from the joined GHASH parts; then the
// frame's chunk headers walked (snap_walk's size pass) and the chunks
// decoded on every thread; the plaintext buffer wiped on every path.  Same
// output and status order as ecies_decrypt_snap, which it falls back to.
// key / key_eph: a key already derived (ecies_derive_key) for the ephemeral
// public key key_eph, used when the envelope's own equals it.
int ecies_decrypt_snap_par(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n,
                           uint8_t *out, uint64_t cap, uint64_t *out_len, const uint8_t *key = nullptr,
                           const uint8_t *key_eph = nullptr);
// ecies_encrypt / ecies_decrypt (no snappy) for one object of at least
// STAGE_PAR_MIN bytes with AES-GCM split over the same pool; same output and
// statuses (a short buffer, a small object or a busy pool: the one-thread
// functions).  On a bad tag the written plaintext is wiped.
int ecies_encrypt_par_plain(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk,
                            const uint8_t *nonce, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                            uint64_t *out_len);
int ecies_decrypt_par(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                      uint64_t cap, uint64_t *out_len, const uint8_t *key = nullptr,
                      const uint8_t *key_eph = nullptr);
// snap_compress / snap_decompress for one object of at least STAGE_PAR_MIN
// bytes on the same pool: the 64 KiB blocks compressed (or the frame's
// chunks decoded) on every thread; same bytes and statuses (a smaller object,
// a short buffer or a busy pool: the one-thread functions).
int snap_compress_par(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
int snap_decompress_par(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len);
// An envelope of n bytes is decrypted on the pool (ecies_decrypt_par /
// ecies_decrypt_snap_par) unless the pool is busy: at least STAGE_PAR_MIN of
// ciphertext, within GCM's length limit, on the VAES path.  (A key derived
// ahead, ecies_derive_key, is used by the pool and the one-thread paths alike.)
bool ecies_par_eligible(uint64_t n);
// f(0) .. f(parts - 1) on the stage pool's threads and the caller, claimed
// one at a time (the caller alone when the pool is busy or single-threaded);
// returns when all are done.  For one object's host copies (api_single.cpp).
void par_for(int parts, const std::function<void(int)> &f);
// The AES key of an envelope whose ephemeral public key (65 B) is eph.
int ecies_derive_key(const uint8_t *secret, uint64_t secret_len, const uint8_t eph[65], uint8_t key[32]);
void secure_wipe(void *p, size_t n);
// the first n bytes of a stream's content from its chunk slots row + coff[i]
void gather_chunks(uint8_t *dst, const uint8_t *row, const uint64_t *coff, uint64_t n);
// the reverse: content bytes [0, n) of src into their chunk slots row + coff[i]
void gather_chunks_to_slots(uint8_t *row, const uint64_t *coff, const uint8_t *src, uint64_t n);

}  // namespace host
}  // namespace chip
