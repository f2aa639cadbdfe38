// host_stages.cpp — ECIES for the host side of encode()/decode()
// (encoding.rs:30-36 `ecies`; decoding.rs:62-77), and the one-pass stages
// that run it together with the snappy framing of host_snap.cpp.
//
// ECIES: ecies 0.2.6 with its default config — receiver key parsed from 33 or
// 65 bytes, ephemeral secp256k1 key, shared point = receiver * ephemeral,
// key = HKDF-SHA256(salt = none, ikm = eph_pub65 || shared65, info = none),
// AES-256-GCM with a 16-byte nonce and no AAD; output
// eph_pub65 || nonce16 || tag16 || ciphertext.  Scalar multiplications in
// secp256k1_host.hpp, AES-GCM in gcm_vaes.cpp (OpenSSL's EVP where the CPU
// lacks VAES), hashes and point parsing from OpenSSL 3 libcrypto; both values
// the reference draws from its RNG can be injected for bit-exact tests.
#include "host_stages.hpp"
#include "gcm_vaes.hpp"
#include "secp256k1_host.hpp"
#include "snap_internal.hpp"

#include <openssl/crypto.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/rand.h>

#include <immintrin.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/carbonado_hip.h"

#pragma GCC diagnostic ignored "-Wdeprecated-declarations"

namespace chip {
namespace host {

// ---------------------------------------------------------------- ECIES
namespace {

struct EcCtx {
    EC_GROUP *g = nullptr;
    BN_CTX *bn = nullptr;
    EcCtx() {
        g = EC_GROUP_new_by_curve_name(NID_secp256k1);
        bn = BN_CTX_new();
    }
    ~EcCtx() {
        BN_CTX_free(bn);
        EC_GROUP_free(g);
    }
};

EcCtx &ec() {
    thread_local EcCtx c;
    return c;
}

struct BnPtr {
    BIGNUM *p;
    explicit BnPtr(BIGNUM *x) : p(x) {}
    ~BnPtr() { BN_clear_free(p); }
};
struct PtPtr {
    EC_POINT *p;
    explicit PtPtr(EC_POINT *x) : p(x) {}
    ~PtPtr() { EC_POINT_free(p); }
};

// libsecp256k1 SecretKey::parse: 32 bytes, 0 < k < n
BIGNUM *parse_secret(const uint8_t *sk, uint64_t len) {
    if (len != 32) return nullptr;
    BIGNUM *k = BN_bin2bn(sk, 32, nullptr);
    if (!k) return nullptr;
    if (BN_is_zero(k) || BN_cmp(k, EC_GROUP_get0_order(ec().g)) >= 0) {
        BN_clear_free(k);
        return nullptr;
    }
    return k;
}

// libsecp256k1 PublicKey::parse_slice(.., None): 33 (compressed), 64 (raw x||y) or 65 bytes
EC_POINT *parse_public(const uint8_t *pk, uint64_t len) {
    uint8_t buf[65];
    const uint8_t *p = pk;
    size_t l = (size_t)len;
    if (len == 64) {
        buf[0] = 0x04;
        std::memcpy(buf + 1, pk, 64);
        p = buf;
        l = 65;
    } else if (len != 33 && len != 65) {
        return nullptr;
    }
    EC_POINT *pt = EC_POINT_new(ec().g);
    if (!pt) return nullptr;
    if (EC_POINT_oct2point(ec().g, pt, p, l, ec().bn) != 1 || EC_POINT_is_at_infinity(ec().g, pt)) {
        EC_POINT_free(pt);
        return nullptr;
    }
    return pt;
}

// OpenSSL 3 looks an algorithm up in its provider store (under a global
// lock) on every init through EVP_sha256() / aes256_gcm() and every
// one-shot HMAC(); the per-object inits of a 16-thread batch serialised on
// it.  Fetched once here, each init only takes a reference.
const EVP_MD *sha256_md() {
    static EVP_MD *m = EVP_MD_fetch(nullptr, "SHA2-256", nullptr);
    return m;
}
const EVP_CIPHER *aes256_gcm() {
    static EVP_CIPHER *c = EVP_CIPHER_fetch(nullptr, "AES-256-GCM", nullptr);
    return c;
}

struct MdCtx {
    EVP_MD_CTX *m = EVP_MD_CTX_new();
    ~MdCtx() { EVP_MD_CTX_free(m); }
};

// HMAC-SHA256 with a 32-byte key (RFC 2104: the key zero-padded to the
// 64-byte block): H((K ^ opad) || H((K ^ ipad) || msg))
bool hmac_sha256_k32(const uint8_t key[32], const uint8_t *msg, size_t n, uint8_t out[32]) {
    thread_local MdCtx ctx;
    EVP_MD_CTX *m = ctx.m;
    uint8_t pad[64], inner[32];
    for (int i = 0; i < 64; ++i) pad[i] = (uint8_t)((i < 32 ? key[i] : 0) ^ 0x36);
    unsigned int l = 0;
    bool ok = m && EVP_DigestInit_ex2(m, sha256_md(), nullptr) == 1 && EVP_DigestUpdate(m, pad, 64) == 1 &&
              EVP_DigestUpdate(m, msg, n) == 1 && EVP_DigestFinal_ex(m, inner, &l) == 1 && l == 32;
    for (int i = 0; i < 64; ++i) pad[i] = (uint8_t)((i < 32 ? key[i] : 0) ^ 0x5c);
    ok = ok && EVP_DigestInit_ex2(m, sha256_md(), nullptr) == 1 && EVP_DigestUpdate(m, pad, 64) == 1 &&
         EVP_DigestUpdate(m, inner, 32) == 1 && EVP_DigestFinal_ex(m, out, &l) == 1 && l == 32;
    OPENSSL_cleanse(pad, sizeof pad);
    OPENSSL_cleanse(inner, sizeof inner);
    return ok;
}

// HKDF-SHA256 (RFC 5869) with no salt and no info, 32-byte output: one HMAC
// for the extract step, one for T(1).
bool hkdf_sha256_32(const uint8_t *ikm, size_t n, uint8_t out[32]) {
    const uint8_t zero[32] = {0}, one = 0x01;
    uint8_t prk[32];
    const bool ok = hmac_sha256_k32(zero, ikm, n, prk) && hmac_sha256_k32(prk, &one, 1, out);
    OPENSSL_cleanse(prk, 32);
    return ok;
}

// k * G as 0x04 || x || y (secp256k1_host.hpp: constant time, ~25x OpenSSL's
// generic ladder for this curve)
bool mul_g65(const BIGNUM *k, uint8_t out[65]) {
    uint8_t kb[32];
    if (BN_bn2binpad(k, kb, 32) != 32) return false;
    const bool ok = k1::to65(k1::mul_g(kb), out);
    OPENSSL_cleanse(kb, sizeof kb);
    return ok;
}

// encapsulate / decapsulate: key = HKDF(eph_pub65 || (peer * secret)65).  The
// peer was parsed and checked to lie on the curve by OpenSSL (parse_public).
bool derive_key(const BIGNUM *secret, const EC_POINT *peer, const uint8_t eph_pub[65], uint8_t key[32]) {
    uint8_t kb[32], xb[32], yb[32];
    BnPtr x(BN_new()), y(BN_new());
    if (!x.p || !y.p || EC_POINT_get_affine_coordinates(ec().g, peer, x.p, y.p, ec().bn) != 1 ||
        BN_bn2binpad(x.p, xb, 32) != 32 || BN_bn2binpad(y.p, yb, 32) != 32 || BN_bn2binpad(secret, kb, 32) != 32)
        return false;
    uint8_t master[130];
    std::memcpy(master, eph_pub, 65);
    bool ok = k1::to65(k1::mul(kb, k1::fe_from_be(xb), k1::fe_from_be(yb)), master + 65);
    OPENSSL_cleanse(kb, sizeof kb);
    ok = ok && hkdf_sha256_32(master, 130, key);
    OPENSSL_cleanse(master, sizeof master);
    return ok;
}

struct CipherCtx {
    const bool fast = gcm_vaes_on();
    bool enc = true;
    EVP_CIPHER_CTX *c = fast ? nullptr : EVP_CIPHER_CTX_new();
    Gcm g;
    ~CipherCtx() {
        if (c) EVP_CIPHER_CTX_free(c);
        if (fast) g.wipe();
    }
    bool init(const uint8_t key[32], const uint8_t iv[16], bool encrypt) {
        enc = encrypt;
        if (fast) {
            g.init(key, iv, 16, encrypt);
            return true;
        }
        if (!c) return false;
        if (encrypt)
            return EVP_EncryptInit_ex(c, aes256_gcm(), nullptr, nullptr, nullptr) == 1 &&
                   EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 16, nullptr) == 1 &&
                   EVP_EncryptInit_ex(c, nullptr, nullptr, key, iv) == 1;
        return EVP_DecryptInit_ex(c, aes256_gcm(), nullptr, nullptr, nullptr) == 1 &&
               EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 16, nullptr) == 1 &&
               EVP_DecryptInit_ex(c, nullptr, nullptr, key, iv) == 1;
    }
    // any length (EVP takes int lengths: fed in 1 GiB steps)
    bool update(const uint8_t *in, uint64_t n, uint8_t *out) {
        if (fast) return g.update(in, n, out);
        constexpr uint64_t STEP = 1ull << 30;
        for (uint64_t o = 0; o < n; o += STEP) {
            const int len = (int)((n - o) < STEP ? (n - o) : STEP);
            int got = 0;
            const int ok = enc ? EVP_EncryptUpdate(c, out + o, &got, in + o, len)
                               : EVP_DecryptUpdate(c, out + o, &got, in + o, len);
            if (ok != 1 || got != len) return false;
        }
        return true;
    }
    // encrypt: the tag of the message
    bool tag(uint8_t out[16]) {
        if (fast) {
            g.tag(out);
            return true;
        }
        int fin = 0;
        uint8_t none[16];  // GCM's final step emits no bytes
        return EVP_EncryptFinal_ex(c, none, &fin) == 1 && fin == 0 &&
               EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out) == 1;
    }
    // decrypt: true when the message's tag equals `want`
    bool check(const uint8_t want[16]) {
        if (fast) {
            uint8_t t[16];
            g.tag(t);
            const bool ok = CRYPTO_memcmp(t, want, 16) == 0;
            OPENSSL_cleanse(t, 16);
            return ok;
        }
        uint8_t w[16], none[16];
        std::memcpy(w, want, 16);
        int fin = 0;
        return EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, w) == 1 && EVP_DecryptFinal_ex(c, none, &fin) == 1;
    }
};

}  // namespace

// AES-256-GCM with a 16-byte nonce and no additional data: the VAES path
// (gcm_vaes.cpp) where the CPU has it, else OpenSSL's EVP (CHIP_GCM=openssl
// forces it; same bytes and tags either way).
bool gcm_vaes_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_GCM");
        return gcm_fast_available() && !(v && std::strcmp(v, "openssl") == 0);
    }();
    return on;
}

int ecies_public_key(const uint8_t *secret, uint8_t out[65]) {
    BnPtr k(parse_secret(secret, 32));
    if (!k.p) return CHIP_ERR_ECIES;
    if (!mul_g65(k.p, out)) return CHIP_ERR_ECIES;
    return CHIP_OK;
}

int ecies_peer(const uint8_t *pubkey, uint64_t pubkey_len, uint8_t peer[65]) {
    if (pubkey_len == 33) {  // compressed: the square root in secp256k1_host.hpp (OpenSSL's BN route: ~27 us)
        k1::Fe x, y;
        if (!pubkey || !k1::decompress(pubkey, x, y)) return CHIP_ERR_ECIES;
        peer[0] = 0x04;
        k1::fe_to_be(x, peer + 1);
        k1::fe_to_be(y, peer + 33);
        return CHIP_OK;
    }
    if (pubkey && (pubkey_len == 64 || (pubkey_len == 65 && pubkey[0] == 0x04))) {  // uncompressed / raw x || y
        peer[0] = 0x04;
        std::memcpy(peer + 1, pubkey + (pubkey_len - 64), 64);
        k1::Fe x, y;
        return k1::parse_full(peer, x, y) ? CHIP_OK : CHIP_ERR_ECIES;
    }
    PtPtr pt(parse_public(pubkey, pubkey_len));
    if (!pt.p) return CHIP_ERR_ECIES;
    BnPtr x(BN_new()), y(BN_new());
    if (!x.p || !y.p || EC_POINT_get_affine_coordinates(ec().g, pt.p, x.p, y.p, ec().bn) != 1 ||
        BN_bn2binpad(x.p, peer + 1, 32) != 32 || BN_bn2binpad(y.p, peer + 33, 32) != 32)
        return CHIP_ERR_ECIES;
    peer[0] = 0x04;
    return CHIP_OK;
}

// 0 < k < n (libsecp256k1 SecretKey::parse), without BIGNUM arithmetic
static bool scalar_ok(const uint8_t k[32]) {
    uint64_t x[4];
    for (int i = 0; i < 4; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w = (w << 8) | k[(3 - i) * 8 + j];
        x[i] = w;
    }
    unsigned long long t;
    unsigned char b = _subborrow_u64(0, x[0], k1::N0, &t);
    b = _subborrow_u64(b, x[1], k1::N1, &t);
    b = _subborrow_u64(b, x[2], k1::N2, &t);
    b = _subborrow_u64(b, x[3], k1::N3, &t);
    return b && (x[0] | x[1] | x[2] | x[3]) != 0;
}

// sk * peer for an encryption's receiver key.  A storage client encrypts
// segment after segment for one receiver, so a key seen before gets a comb
// table of its own (k1::CombTable, built on its second use outside the lock,
// ~0.3 ms, at most 8 receivers kept, 123 KB each): the ECDH then costs what
// k * G does instead of the GLV ladder's 132 doublings.  The table is public
// data (multiples of a public key); the scalar is used exactly as in mul_g
// (full table scans, fixed step count: the same constant-time code).
// CHIP_PEER_TABLES=0 turns it off.
static k1::Pt peer_mul(const uint8_t peer[65], const uint8_t sk[32]) {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_PEER_TABLES");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    const k1::Fe px = k1::fe_from_be(peer + 1), py = k1::fe_from_be(peer + 33);
    if (!on) return k1::mul(sk, px, py);
    struct Entry {
        uint8_t key[64];
        uint32_t uses = 0;
        uint64_t stamp = 0;
        std::shared_ptr<const k1::CombTable> table;
        bool building = false;
    };
    static std::mutex mu;
    static Entry cache[8];
    static uint64_t clock = 0;
    std::shared_ptr<const k1::CombTable> table;
    Entry *e = nullptr;
    bool build = false;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (Entry &x : cache)
            if (x.uses && std::memcmp(x.key, peer + 1, 64) == 0) e = &x;
        if (!e) {  // a new receiver replaces the least recently used one
            e = &cache[0];
            for (Entry &x : cache)
                if (!x.building && x.stamp < e->stamp) e = &x;
            if (e->building) e = nullptr;  // every slot busy building: no table this time
            else {
                *e = Entry{};
                std::memcpy(e->key, peer + 1, 64);
            }
        }
        if (e) {
            e->stamp = ++clock;
            ++e->uses;
            table = e->table;
            if (!table && e->uses >= 2 && !e->building) build = e->building = true;
        }
    }
    if (build) {
        auto t = std::make_shared<const k1::CombTable>(px, py);
        std::lock_guard<std::mutex> lk(mu);
        if (std::memcmp(e->key, peer + 1, 64) == 0) e->table = t;  // (not replaced meanwhile)
        e->building = false;
        table = t;
    }
    return table ? k1::mul_comb(*table, sk) : k1::mul(sk, px, py);
}

int ecies_prepare(const uint8_t peer[65], const uint8_t *eph_sk, EciesKey *out) {
    // the two scalar multiplications side by side (a stage-pool worker takes
    // one unless the pool is busy: then both here, one after the other)
    return ecies_prepare_with(peer, eph_sk, out, [](const std::function<void(int)> &f) { par_for(2, f); });
}

int ecies_prepare_with(const uint8_t peer[65], const uint8_t *eph_sk, EciesKey *out,
                       const std::function<void(const std::function<void(int)> &)> &run2) {
    uint8_t sk[32];
    if (eph_sk) {
        std::memcpy(sk, eph_sk, 32);
        if (!scalar_ok(sk)) return CHIP_ERR_ECIES;
    } else {
        do {  // SecretKey::random: rejection-sample a valid scalar
            if (RAND_bytes(sk, 32) != 1) return CHIP_ERR_ECIES;
        } while (!scalar_ok(sk));
    }
    uint8_t master[130];
    k1::Pt pts[2];
    run2([&](int i) { pts[i] = i == 0 ? k1::mul_g(sk) : peer_mul(peer, sk); });
    bool ok = k1::to65_pair(pts[0], pts[1], out->eph_pub, master + 65);
    std::memcpy(master, out->eph_pub, 65);
    OPENSSL_cleanse(sk, sizeof sk);
    ok = ok && hkdf_sha256_32(master, 130, out->key);
    OPENSSL_cleanse(master, sizeof master);
    return ok ? CHIP_OK : CHIP_ERR_ECIES;
}

void ecies_key_wipe(EciesKey *k) { OPENSSL_cleanse(k, sizeof *k); }

// Header and cipher context from prepared key material (ecies_prepare).
static int ecies_begin_prepared(const EciesKey &k, const uint8_t *nonce, uint8_t *out, CipherCtx &cc) {
    std::memcpy(out, k.eph_pub, 65);
    uint8_t *iv = out + 65;
    if (nonce) std::memcpy(iv, nonce, 16);
    else if (RAND_bytes(iv, 16) != 1) return CHIP_ERR_ECIES;
    return cc.init(k.key, iv, true) ? CHIP_OK : CHIP_ERR_ECIES;
}

// ECIES header (ephemeral public key, nonce) into out[0, 81) and the
// AES-256-GCM context keyed for the ciphertext at out + 97; the tag goes to
// out[81, 97) when the ciphertext is done.
static int ecies_begin(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                       uint8_t *out, CipherCtx &cc) {
    uint8_t peer[65];
    EciesKey k;
    int st = ecies_peer(pubkey, pubkey_len, peer);
    if (st == CHIP_OK) st = ecies_prepare(peer, eph_sk, &k);
    if (st == CHIP_OK) st = ecies_begin_prepared(k, nonce, out, cc);
    ecies_key_wipe(&k);
    return st;
}

static int ecies_end(CipherCtx &cc, uint8_t *out, uint64_t ct_len, uint64_t *out_len) {
    if (!cc.tag(out + 81)) return CHIP_ERR_ECIES;
    *out_len = ct_len + ECIES_OVERHEAD;
    return CHIP_OK;
}

int ecies_encrypt(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                  const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (cap < n + ECIES_OVERHEAD) return CHIP_ERR_BUFFER_TOO_SMALL;
    CipherCtx cc;
    int st = ecies_begin(pubkey, pubkey_len, eph_sk, nonce, out, cc);
    if (st != CHIP_OK) return st;
    if (!cc.update(in, n, out + 97)) return CHIP_ERR_ECIES;
    return ecies_end(cc, out, n, out_len);
}


// The AES key of an envelope whose ephemeral public key is eph (65 B as the
// envelope holds it) for the receiver's secret (32 B, 0 < k < n: checked by
// the caller): the usual uncompressed form parsed and checked here
// (k1::parse_full; OpenSSL's BIGNUM route cost ~30 us more per call), the
// hybrid 0x06 / 0x07 forms through OpenSSL; then HKDF(eph || (k * eph)65).
static bool eph_key(const uint8_t secret[32], const uint8_t eph[65], uint8_t key[32]) {
    if (eph[0] != 0x04) {
        BnPtr k(parse_secret(secret, 32));
        PtPtr pt(parse_public(eph, 65));
        return k.p && pt.p && derive_key(k.p, pt.p, eph, key);
    }
    k1::Fe x, y;
    if (!k1::parse_full(eph, x, y)) return false;
    uint8_t master[130];
    std::memcpy(master, eph, 65);
    bool ok = k1::to65(k1::mul(secret, x, y), master + 65);
    ok = ok && hkdf_sha256_32(master, 130, key);
    OPENSSL_cleanse(master, sizeof master);
    return ok;
}

// the envelope's AES key: the one derived ahead when its ephemeral key is
// this envelope's, else from the secret and the envelope's ephemeral key
static bool envelope_key(const uint8_t *secret, const uint8_t *in, const uint8_t *pre_key, const uint8_t *pre_eph,
                         uint8_t key[32]) {
    if (pre_key && pre_eph && std::memcmp(pre_eph, in, 65) == 0) {
        std::memcpy(key, pre_key, 32);
        return true;
    }
    return eph_key(secret, in, key);
}

int ecies_decrypt(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                  uint64_t cap, uint64_t *out_len, const uint8_t *pre_key, const uint8_t *pre_eph) {
    if (!secret || secret_len != 32 || !scalar_ok(secret)) return CHIP_ERR_ECIES;  // SecretKey::parse
    if (n < ECIES_OVERHEAD) return CHIP_ERR_ECIES;  // InvalidMessage
    const uint64_t m = n - ECIES_OVERHEAD;
    if (cap < m || (m && !out)) {
        *out_len = m;
        return CHIP_ERR_BUFFER_TOO_SMALL;
    }
    uint8_t key[32];
    if (!envelope_key(secret, in, pre_key, pre_eph, key)) return CHIP_ERR_ECIES;
    const uint8_t *iv = in + 65, *tag = in + 81, *ct = in + 97;
    CipherCtx cc;
    bool ok = cc.init(key, iv, false) && cc.update(ct, m, out);
    OPENSSL_cleanse(key, 32);
    ok = ok && cc.check(tag);
    if (!ok) {
        if (m) OPENSSL_cleanse(out, m);  // never hand back unauthenticated plaintext
        return CHIP_ERR_ECIES;
    }
    *out_len = m;
    return CHIP_OK;
}

// Ecies|Snappy decode in one pass.  The two-pass form writes the whole
// plaintext to a scratch buffer and reads it back for the snappy walk: two
// extra DRAM passes per object, and level-15 decode end to end is bound by
// the host threads' memory traffic beside the DMA.  Here the
// plaintext is decrypted into a per-thread window of 256 KiB (L2-resident)
// and each snappy chunk is decoded from there into `out`.  Status order equals
// ecies_decrypt + snap_decompress: a bad tag is EciesError whatever the
// plaintext holds; then framing errors (snap_walk's size pass); then a short
// `out` (required size in *out_len); then CRC / block errors.  A data chunk
// longer than the window (never produced by a FrameEncoder) takes the
// two-pass route.
int ecies_decrypt_snap(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                       uint64_t cap, uint64_t *out_len, uint8_t *window, const uint8_t *pre_key,
                       const uint8_t *pre_eph) {
    if (!secret || secret_len != 32 || !scalar_ok(secret)) return CHIP_ERR_ECIES;  // SecretKey::parse
    if (n < ECIES_OVERHEAD) return CHIP_ERR_ECIES;
    const uint64_t m = n - ECIES_OVERHEAD;
    uint8_t key[32];
    if (!envelope_key(secret, in, pre_key, pre_eph, key)) return CHIP_ERR_ECIES;
    const uint8_t *iv = in + 65, *ct = in + 97;
    const uint8_t *tag = in + 81;
    CipherCtx cc;
    bool dec_ok = cc.init(key, iv, false);
    OPENSSL_cleanse(key, 32);
    if (!dec_ok) return CHIP_ERR_ECIES;

    constexpr uint64_t W = DECRYPT_SNAP_WINDOW;
    static thread_local std::unique_ptr<uint8_t[]> t_win;
    if (!window && !t_win) t_win.reset(new uint8_t[W]);
    uint8_t *win = window ? window : t_win.get();
    uint64_t wbeg = 0, wend = 0;  // plaintext [wbeg, wend) sits at win[0 .. wend - wbeg)
    // plaintext [s, s + len) resident in the window; s only moves forward,
    // len <= W and s + len <= m
    auto need = [&](uint64_t s, uint64_t len) -> const uint8_t * {
        if (s + len <= wend) return win + (s - wbeg);
        uint64_t keep = 0;
        if (s < wend) {
            keep = wend - s;
            std::memmove(win, win + (s - wbeg), keep);
        }
        while (wend < s) {  // a skipped chunk: decrypted (for the tag) and dropped
            const uint64_t step = std::min<uint64_t>(W, s - wend);
            dec_ok &= cc.update(ct + wend, step, win);
            wend += step;
        }
        wbeg = s;
        wend = s + keep;
        const uint64_t step = std::min<uint64_t>(W - keep, m - wend);
        dec_ok &= cc.update(ct + wend, step, win + keep);
        wend += step;
        return win;
    };

    uint64_t s = 0, d = 0;
    const uint64_t ecap = out ? cap : 0;  // no buffer: size the output, write nothing
    bool ident = false, fits = true, two_pass = false;
    int frame = CHIP_OK, content = CHIP_OK;
    while (s < m) {  // snap_walk's chunk loop, both passes at once
        if (m - s < 4) { frame = CHIP_ERR_SNAP; break; }
        const uint8_t *h = need(s, 4);
        const uint8_t ty = h[0];
        const uint64_t clen = (uint64_t)h[1] | ((uint64_t)h[2] << 8) | ((uint64_t)h[3] << 16);
        s += 4;
        if (clen > m - s) { frame = CHIP_ERR_SNAP; break; }
        if (!ident && ty != 0xFF) { frame = CHIP_ERR_SNAP; break; }
        if (ty >= 0x02 && ty <= 0x7F) { frame = CHIP_ERR_SNAP; break; }
        if (ty >= 0x80 && ty != 0xFF) { s += clen; continue; }  // skippable
        if (clen > W) { two_pass = true; break; }
        const uint8_t *body = need(s, clen);
        if (ty == 0xFF) {
            if (clen != 6 || std::memcmp(body, STREAM_ID + 4, 6) != 0) { frame = CHIP_ERR_SNAP; break; }
            ident = true;
        } else {
            if (clen < 4) { frame = CHIP_ERR_SNAP; break; }
            uint32_t want;
            std::memcpy(&want, body, 4);
            const uint8_t *data = body + 4;
            const uint64_t dl = clen - 4;
            uint64_t ulen = dl;
            if (ty == 0x01) {
                if (dl > MAX_BLOCK) { frame = CHIP_ERR_SNAP; break; }
            } else {
                size_t used;
                if (!get_varint(data, dl, &ulen, &used) || ulen > MAX_BLOCK) { frame = CHIP_ERR_SNAP; break; }
            }
            if (fits && ulen > ecap - d) fits = false;
            if (fits && content == CHIP_OK) {
                if (ty == 0x01) {
                    if (crc_masked(data, dl) != want) content = CHIP_ERR_SNAP;
                    else std::memcpy(out + d, data, dl);
                } else {
                    size_t got;
                    if (!decompress_raw(data, dl, out + d, ulen, &got) || got != ulen ||
                        crc_masked(out + d, ulen) != want)
                        content = CHIP_ERR_SNAP;
                }
            }
            d += ulen;
        }
        s += clen;
    }
    if (two_pass) {
        // what was written so far is not authenticated yet: wipe it (and the
        // window) before the two-pass route, whose decrypt checks the tag first
        if (d && out) OPENSSL_cleanse(out, std::min(d, ecap));
        OPENSSL_cleanse(win, W);
        std::vector<uint8_t> tmp(m + 1);
        uint64_t got = 0;
        int st = ecies_decrypt(secret, secret_len, in, n, tmp.data(), tmp.size(), &got, pre_key, pre_eph);
        if (st == CHIP_OK) st = snap_decompress(tmp.data(), got, out, cap, out_len);
        OPENSSL_cleanse(tmp.data(), tmp.size());
        return st;
    }
    while (wend < m) {  // the rest of the ciphertext, for the tag
        const uint64_t step = std::min<uint64_t>(W, m - wend);
        dec_ok &= cc.update(ct + wend, step, win);
        wend += step;
    }
    dec_ok = dec_ok && cc.check(tag);
    OPENSSL_cleanse(win, W);
    if (!dec_ok) {
        if (d && out) OPENSSL_cleanse(out, std::min(d, ecap));  // never hand back unauthenticated plaintext
        return CHIP_ERR_ECIES;
    }
    if (frame != CHIP_OK) return frame;
    if (!fits || (d && !out)) {
        *out_len = d;
        return CHIP_ERR_BUFFER_TOO_SMALL;
    }
    if (content != CHIP_OK) return content;
    *out_len = d;
    return CHIP_OK;
}

namespace {

bool nt_copy_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_NT_COPY");
        if (v && v[0] == '0' && v[1] == 0) return false;
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx2") != 0;
    }();
    return on;
}

__attribute__((target("avx2"))) void nt_copy_avx2(uint8_t *d, const uint8_t *s, size_t n, bool fence = true) {
    size_t head = (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31;
    if (head > n) head = n;
    std::memcpy(d, s, head);
    size_t i = head;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 96), e);
    }
    for (; i + 32 <= n; i += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i)));
    std::memcpy(d + i, s + i, n - i);
    if (fence) _mm_sfence();  // the streaming stores are globally visible before the DMA is enqueued
}

}  // namespace

void ring_copy(void *dst, const void *src, size_t n) {
    if (n >= 4096 && nt_copy_on()) nt_copy_avx2(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
    else std::memcpy(dst, src, n);
}

// one 1024-B chunk into its stream slot (8 mod 64): the whole lines with
// streaming stores, the two partial ones (shared with parent nodes / the
// device-copied tail) with plain stores; the caller fences once
__attribute__((target("avx2"))) static void chunk_nt(uint8_t *d, const uint8_t *s) {
    const size_t head = (64 - (reinterpret_cast<uintptr_t>(d) & 63)) & 63;
    std::memcpy(d, s, head);
    size_t i = head;
    for (; i + 64 <= 1024; i += 64) {
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i)));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32),
                            _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32)));
    }
    std::memcpy(d + i, s + i, 1024 - i);
}

__attribute__((target("avx2"))) static void fence_nt() { _mm_sfence(); }

void fill_data_chunks(uint8_t *out, const uint64_t *coff, uint64_t nd, uint64_t zl, const uint8_t *src, uint64_t n) {
    for (int b = 0; b < 8; ++b) out[b] = static_cast<uint8_t>(zl >> (8 * b));  // bao header: u64 LE length
    fill_chunk_range(out, coff, 0, nd, src, n);
}

void fill_chunk_range(uint8_t *out, const uint64_t *coff, uint64_t c0, uint64_t c1, const uint8_t *src, uint64_t n) {
    const bool nt = nt_copy_on();
    alignas(64) uint8_t pad[1024];
    for (uint64_t i = c0; i < c1; ++i) {
        const uint64_t off = 1024 * i;
        const uint8_t *s = src + (off < n ? off : 0);
        if (off + 1024 > n) {  // the zfec padding: zeros past the input
            const uint64_t v = off < n ? n - off : 0;
            if (v) std::memcpy(pad, s, v);
            std::memset(pad + v, 0, 1024 - v);
            s = pad;
        }
        if (nt) chunk_nt(out + coff[i], s);
        else std::memcpy(out + coff[i], s, 1024);
    }
    if (nt) fence_nt();
}

bool nt_stage_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_NT_STAGE");
        return !(v && v[0] == '0' && v[1] == 0) && nt_copy_on();
    }();
    return on;
}

namespace {

// The ECIES output as it is produced, cut into the 1024-B chunks of the
// Zfec|Bao stream it becomes: whole chunks [1, nd) go to their slots, a chunk
// split across two blocks is assembled in `part`; chunk 0 (which holds the
// tag) is kept in `first` until finish().  `pos` = output offset of the next
// byte pushed.
struct ChunkAssembler {
    const ChunkSink *sink;
    bool nt;
    uint64_t hl = 97;  // bytes of a header written last (ECIES: key, nonce, tag); 0 for a snappy frame
    uint64_t pos = hl;
    alignas(64) uint8_t part[1024];
    alignas(64) uint8_t first[1024];
    void slot(uint64_t ci, const uint8_t *src) {
        if (nt) chunk_nt(sink->out + sink->coff[ci], src);
        else std::memcpy(sink->out + sink->coff[ci], src, 1024);
    }
    void push(const uint8_t *p, size_t len) {
        while (len) {
            const uint64_t ci = pos / 1024, at = pos % 1024;
            const size_t take = (size_t)std::min<uint64_t>(len, 1024 - at);
            if (ci == 0 && hl) {
                std::memcpy(first + at, p, take);
            } else if (ci < sink->nd) {
                if (at == 0 && take == 1024) {
                    slot(ci, p);
                } else {
                    std::memcpy(part + at, p, take);
                    if (at + take == 1024) slot(ci, part);
                }
            }
            p += take;
            len -= take;
            pos += take;
        }
    }
    // chunks placed: [1, done()) with a held header, [0, done()) without
    uint64_t done() const {
        const uint64_t c = std::min<uint64_t>(sink->nd, pos / 1024);
        return hl ? std::max<uint64_t>(1, c) : c;
    }
    // the rest of the output's chunks: the stream header, chunk 0 (with a
    // held header: it + the first bytes after it) and the last partial chunk,
    // zero padded; returns the chunks placed ([0, ceil(pos / 1024)))
    uint64_t finish(const uint8_t *head) {
        for (int b = 0; b < 8; ++b) sink->out[b] = static_cast<uint8_t>(sink->zl >> (8 * b));
        if (hl) {
            std::memcpy(first, head, hl);
            if (pos < 1024) std::memset(first + pos, 0, 1024 - pos);
            slot(0, first);
        }
        if (pos % 1024 && (pos > 1024 || !hl)) {
            std::memset(part + pos % 1024, 0, 1024 - pos % 1024);
            slot(pos / 1024, part);
        }
        return (pos + 1023) / 1024;
    }
};

}  // namespace

// window halves: snap_block's compression scratch, then one block's frame piece
static_assert(SNAP_ECIES_WINDOW / 2 >= MAX_COMPRESS_BLOCK && SNAP_ECIES_WINDOW / 2 >= 8 + MAX_BLOCK,
              "SNAP_ECIES_WINDOW too small");

int ecies_encrypt_stream(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                         const uint8_t *in, uint64_t n, bool snap, uint8_t *out, uint64_t cap, uint64_t *out_len,
                         uint8_t *window, const ChunkSink *sink, uint64_t *filled, const EciesKey *prepared) {
    const uint64_t m = snap ? snap_max_len(n) : n;
    if (out && cap < m + ECIES_OVERHEAD) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (!out && !(sink && sink->complete)) return CHIP_ERR_INVALID_ARG;
    if (sink && sink->complete && (sink->nd < 1 || 1024 * sink->nd < m + ECIES_OVERHEAD)) return CHIP_ERR_INVALID_ARG;
    if (filled) *filled = 0;
    uint8_t head[97];
    uint8_t *hdr = out ? out : head;
    CipherCtx cc;
    int st = prepared ? ecies_begin_prepared(*prepared, nonce, hdr, cc)
                      : ecies_begin(pubkey, pubkey_len, eph_sk, nonce, hdr, cc);
    if (st != CHIP_OK) return st;
    uint8_t *ct = out ? out + 97 : nullptr;
    uint8_t *piece = window + SNAP_ECIES_WINDOW / 2;  // one block's ciphertext (the sink path)
    const bool nt = sink && nt_stage_on();
    ChunkAssembler as{sink, nt_copy_on()};
    uint64_t off = 0;  // ciphertext bytes so far
    if (snap && n) {
        uint8_t *d = sink ? piece : ct;
        if (!cc.update(STREAM_ID, sizeof(STREAM_ID), d)) return CHIP_ERR_ECIES;
        if (sink) {
            if (ct) std::memcpy(ct, piece, sizeof(STREAM_ID));
            as.push(piece, sizeof(STREAM_ID));
        }
        off = sizeof(STREAM_ID);
    }
    for (uint64_t o = 0; o < n; o += MAX_BLOCK) {
        const size_t len = (size_t)((n - o) < MAX_BLOCK ? (n - o) : MAX_BLOCK);
        // the block's ciphertext: straight into out, or (sink) into the cache-resident
        // piece buffer, from which it is cut into chunks (and streamed to out, if any)
        uint8_t *dst = sink ? piece : ct + off;
        size_t plen;
        if (snap) {
            uint8_t bh[8];
            const uint8_t *body;
            const size_t blen = snap_block(in + o, len, bh, window, &body);
            if (!cc.update(bh, 8, dst) || !cc.update(body, blen, dst + 8))
                return CHIP_ERR_ECIES;
            plen = 8 + blen;
        } else {
            if (!cc.update(in + o, len, dst)) return CHIP_ERR_ECIES;
            plen = len;
        }
        if (sink) {
            if (ct) {
                if (nt) nt_copy_avx2(ct + off, piece, plen, false);
                else std::memcpy(ct + off, piece, plen);
            }
            as.push(piece, plen);
        }
        off += plen;
    }
    st = ecies_end(cc, hdr, off, out_len);
    if (st == CHIP_OK && sink) {
        const uint64_t placed = sink->complete ? as.finish(hdr) : as.done();
        if (filled) *filled = placed;
    }
    if (nt || (sink && as.nt)) fence_nt();
    return st;
}

int snap_compress_stream(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                         uint8_t *window, const ChunkSink *sink, uint64_t *filled) {
    const uint64_t m = snap_max_len(n);
    if (out && cap < m) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (!out && !(sink && sink->complete)) return CHIP_ERR_INVALID_ARG;
    if (sink && sink->complete && 1024 * sink->nd < m) return CHIP_ERR_INVALID_ARG;
    if (filled) *filled = 0;
    *out_len = 0;
    if (n == 0) return CHIP_OK;  // FrameEncoder writes nothing for an empty input
    const bool nt = sink && out && nt_stage_on();
    ChunkAssembler as{sink, nt_copy_on(), 0};
    uint64_t d = 0;
    auto emit = [&](const uint8_t *p, size_t len) {
        if (out) {
            if (nt) nt_copy_avx2(out + d, p, len, false);
            else std::memcpy(out + d, p, len);
        }
        if (sink) as.push(p, len);
        d += len;
    };
    emit(STREAM_ID, sizeof(STREAM_ID));
    for (uint64_t o = 0; o < n; o += MAX_BLOCK) {
        const size_t len = (size_t)((n - o) < MAX_BLOCK ? (n - o) : MAX_BLOCK);
        uint8_t hdr[8];
        const uint8_t *body;
        const size_t blen = snap_block(in + o, len, hdr, window, &body);
        emit(hdr, 8);
        emit(body, blen);
    }
    *out_len = d;
    if (sink) {
        const uint64_t placed = sink->complete ? as.finish(nullptr) : as.done();
        if (filled) *filled = placed;
    }
    if (nt || (sink && as.nt)) fence_nt();
    return CHIP_OK;
}

void secure_wipe(void *p, size_t n) { OPENSSL_cleanse(p, n); }

int ecies_derive_key(const uint8_t *secret, uint64_t secret_len, const uint8_t eph[65], uint8_t key[32]) {
    if (!secret || secret_len != 32 || !scalar_ok(secret)) return CHIP_ERR_ECIES;  // SecretKey::parse
    return eph_key(secret, eph, key) ? CHIP_OK : CHIP_ERR_ECIES;
}

void gather_chunks(uint8_t *dst, const uint8_t *row, const uint64_t *coff, uint64_t n) {
    for (uint64_t i = 0; 1024 * i < n; ++i)
        std::memcpy(dst + 1024 * i, row + coff[i], (size_t)std::min<uint64_t>(1024, n - 1024 * i));
}

void gather_chunks_to_slots(uint8_t *row, const uint64_t *coff, const uint8_t *src, uint64_t n) {
    for (uint64_t i = 0; 1024 * i < n; ++i)
        std::memcpy(row + coff[i], src + 1024 * i, (size_t)std::min<uint64_t>(1024, n - 1024 * i));
}

}  // namespace host
}  // namespace chip
