// gcm_vaes.hpp — AES-256-GCM for the host ECIES stage (ecies 0.2: AES-256-GCM
// with a 16-byte nonce; encoding.rs:31-36, decoding.rs:62-69) on CPUs with
// VAES + VPCLMULQDQ + AVX-512: sixteen blocks per step, the counter blocks
// through four 512-bit AES lanes and their GHASH as four 512-bit carry-less
// products summed before one reduction.  The image's OpenSSL 3.0.2 has no
// such path (its AVX2 form runs 5.5 GiB/s per GPU-box thread, 60 % of the
// level-15 host stage, profiles/r10q_session); host_stages.cpp falls back to
// it where these instructions are missing, or with CHIP_GCM=openssl.
// Byte-for-byte the same output and tags as OpenSSL's EVP AES-256-GCM
// (tests/test_host_stages.py compares them over random keys, nonces,
// lengths and update splits).
#pragma once

#include <cstddef>
#include <cstdint>

namespace chip {
namespace host {

constexpr uint64_t GCM_MAX_BYTES = (1ull << 36) - 32;

// Streaming AES-256-GCM without additional data: init, any number of
// updates of any length, then tag (encrypt) or check (decrypt).
struct Gcm {
    alignas(64) uint8_t rk[15][16];   // AES-256 round keys
    alignas(64) uint8_t hp[16][16];   // H^16 .. H^1, byte-reversed (hp[16 - k] = H^k)
    alignas(16) uint8_t y[16];        // GHASH accumulator, byte-reversed
    uint8_t j0[16];                   // the pre-counter block (tag mask)
    uint8_t prefix[12];               // counter block bytes 0..11
    uint32_t ctr = 0;                 // next counter value (bytes 12..15, big-endian)
    uint8_t ks[16];                   // keystream of the partial block
    uint8_t pend[16];                 // its ciphertext so far (GHASH input)
    uint32_t npend = 0;
    uint64_t len = 0;                 // ciphertext bytes so far
    bool enc = true;

    // key 32 bytes, iv of any nonzero length (ecies: 16)
    void init(const uint8_t *key, const uint8_t *iv, size_t ivlen, bool encrypt);
    // false (nothing processed) once the message would pass GCM's limit of
    // 2^36 - 32 bytes (the 32-bit block counter; OpenSSL refuses it too)
    bool update(const uint8_t *in, size_t n, uint8_t *out);
    void tag(uint8_t out[16]);  // ends the message
    void wipe();

    // One message split over threads: each part is a Gcm made by init_part
    // from the message's Gcm (after init) at a byte offset that is a multiple
    // of 16, fed its bytes with update(), then part_ghash(); the message's
    // Gcm joins every part's GHASH with the number of 16-B blocks of the
    // message after that part, and tag_joined() gives the message's tag.
    void init_part(const Gcm &msg, uint64_t offset);
    void part_ghash(uint8_t out[16]);
    void join_part(const uint8_t y_part[16], uint64_t blocks_after);
    void tag_joined(uint64_t total, uint8_t out[16]);
};

// VAES, VPCLMULQDQ, AVX-512 F/BW/VL, AES-NI and PCLMULQDQ all present
bool gcm_fast_available();
// the ECIES stage uses Gcm (gcm_fast_available() and not CHIP_GCM=openssl;
// host_stages.cpp), else OpenSSL's EVP
bool gcm_vaes_on();

}  // namespace host
}  // namespace chip
