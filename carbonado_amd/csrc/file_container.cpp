// file_container.cpp — the flat-file container around the encoded stream
// (/root/reference/src/file.rs): the 160-byte signed Header and
// file::encode / file::decode.  Host code: the header is 160 bytes per object
// and one BIP-340 signature, nothing for the GPU to do; the body is the
// encode()/decode() path of api_encode.cpp / api_decode.cpp (zfec + bao on
// the device).
//
// Header bytes (Header::try_to_vec, file.rs:292-335):
//   magic "CARBONADO01\n" 12 | pubkey 33 (compressed) | bao hash 32 |
//   Schnorr signature over the hash 64 | format 1 | chunk_index 1 |
//   encoded_len u32 LE | padding_len u32 LE | metadata 8 (zeros = None) | 0
// Signature: BIP-340 (secp256k1 0.28 Keypair::sign_schnorr, file.rs:269-271),
// message = the 32-byte hash, auxiliary randomness from the RNG as the
// reference (thread_rng) or injected for bit-exact tests.  Parsing
// (file.rs:116-154) checks the magic, the pubkey and the signature against the
// x-only pubkey (file.rs:129-131).
#include <openssl/bn.h>
#include <openssl/crypto.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/rand.h>

#include <cstring>
#include <vector>

#include "secp256k1_host.hpp"
#include "../../include/carbonado_hip.h"

namespace {

const uint8_t MAGIC[12] = {'C', 'A', 'R', 'B', 'O', 'N', 'A', 'D', 'O', '0', '1', '\n'};  // constants.rs:4

struct Ctx {
    EC_GROUP *g = nullptr;
    BN_CTX *bn = nullptr;
    BIGNUM *p = nullptr;  // field prime
    Ctx() {
        g = EC_GROUP_new_by_curve_name(NID_secp256k1);
        bn = BN_CTX_new();
        p = BN_new();
        EC_GROUP_get_curve(g, p, nullptr, nullptr, bn);
    }
    ~Ctx() {
        BN_free(p);
        BN_CTX_free(bn);
        EC_GROUP_free(g);
    }
};
// one per thread: BN_CTX is not thread-safe
Ctx &ctx() {
    static thread_local Ctx c;
    return c;
}
const BIGNUM *order() { return EC_GROUP_get0_order(ctx().g); }

struct Bn {
    BIGNUM *v;
    Bn() : v(BN_new()) {}
    explicit Bn(const uint8_t *b32) : v(BN_bin2bn(b32, 32, nullptr)) {}
    ~Bn() { BN_clear_free(v); }
    Bn(const Bn &) = delete;
};
struct Pt {
    EC_POINT *v;
    Pt() : v(EC_POINT_new(ctx().g)) {}
    ~Pt() { EC_POINT_free(v); }
    Pt(const Pt &) = delete;
};

bool sha256(const uint8_t *a, size_t na, const uint8_t *b, size_t nb, const uint8_t *c, size_t nc,
            const uint8_t *d, size_t nd, uint8_t out[32]) {
    EVP_MD_CTX *m = EVP_MD_CTX_new();
    unsigned len = 0;
    bool ok = m && EVP_DigestInit_ex(m, EVP_sha256(), nullptr) == 1 && (!na || EVP_DigestUpdate(m, a, na) == 1) &&
              (!nb || EVP_DigestUpdate(m, b, nb) == 1) && (!nc || EVP_DigestUpdate(m, c, nc) == 1) &&
              (!nd || EVP_DigestUpdate(m, d, nd) == 1) && EVP_DigestFinal_ex(m, out, &len) == 1 && len == 32;
    EVP_MD_CTX_free(m);
    return ok;
}

// BIP-340 tagged hash: SHA256(SHA256(tag) || SHA256(tag) || x || y || z)
bool tagged(const char *tag, const uint8_t *x, size_t nx, const uint8_t *y, size_t ny, const uint8_t *z, size_t nz,
            uint8_t out[32]) {
    uint8_t th[32];
    if (!sha256(reinterpret_cast<const uint8_t *>(tag), std::strlen(tag), nullptr, 0, nullptr, 0, nullptr, 0, th))
        return false;
    EVP_MD_CTX *m = EVP_MD_CTX_new();
    unsigned len = 0;
    bool ok = m && EVP_DigestInit_ex(m, EVP_sha256(), nullptr) == 1 && EVP_DigestUpdate(m, th, 32) == 1 &&
              EVP_DigestUpdate(m, th, 32) == 1 && (!nx || EVP_DigestUpdate(m, x, nx) == 1) &&
              (!ny || EVP_DigestUpdate(m, y, ny) == 1) && (!nz || EVP_DigestUpdate(m, z, nz) == 1) &&
              EVP_DigestFinal_ex(m, out, &len) == 1 && len == 32;
    EVP_MD_CTX_free(m);
    return ok;
}

bool bn32(const BIGNUM *v, uint8_t out[32]) { return BN_bn2binpad(v, out, 32) == 32; }

// affine x (32 B) and whether y is even
bool xy(const EC_POINT *pt, uint8_t x32[32], bool *even) {
    Bn x, y;
    if (EC_POINT_get_affine_coordinates(ctx().g, pt, x.v, y.v, ctx().bn) != 1) return false;
    *even = !BN_is_odd(y.v);
    return bn32(x.v, x32);
}

// k * G (secp256k1_host.hpp: constant time; OpenSSL's generic-curve ladder
// was ~5x slower): affine x and whether y is even
bool mul_g_xy(const BIGNUM *k, uint8_t x32[32], bool *even) {
    uint8_t kb[32], o[65];
    if (!bn32(k, kb)) return false;
    const bool ok = chip::k1::to65(chip::k1::mul_g(kb), o);
    OPENSSL_cleanse(kb, sizeof kb);
    if (!ok) return false;
    std::memcpy(x32, o + 1, 32);
    *even = !(o[64] & 1);
    return true;
}

// a secret key as the reference accepts it (SecretKey::from_slice): 32 bytes, 0 < d < n
bool parse_secret(const uint8_t *sk, uint64_t len, Bn &d) {
    if (!sk || len != 32) return false;
    BN_bin2bn(sk, 32, d.v);
    return !BN_is_zero(d.v) && BN_cmp(d.v, order()) < 0;
}

// PublicKey::from_slice: 33-byte compressed or 65-byte uncompressed point on the curve
bool parse_public(const uint8_t *pk, uint64_t len, Pt &pt) {
    if (!pk || !((len == 33 && (pk[0] == 2 || pk[0] == 3)) || (len == 65 && pk[0] == 4))) return false;
    return EC_POINT_oct2point(ctx().g, pt.v, pk, len, ctx().bn) == 1 && !EC_POINT_is_at_infinity(ctx().g, pt.v) &&
           EC_POINT_is_on_curve(ctx().g, pt.v, ctx().bn) == 1;
}

bool compressed(const EC_POINT *pt, uint8_t out[33]) {
    return EC_POINT_point2oct(ctx().g, pt, POINT_CONVERSION_COMPRESSED, out, 33, ctx().bn) == 33;
}

// BIP-340 lift_x: the point with x and an even y
bool lift_x(const uint8_t x32[32], Pt &pt) {
    Bn x(x32);
    if (BN_cmp(x.v, ctx().p) >= 0) return false;
    return EC_POINT_set_compressed_coordinates(ctx().g, pt.v, x.v, 0, ctx().bn) == 1;
}

// BIP-340 signing.  The key and nonce scalars stay in secp256k1_host.hpp's
// constant-time arithmetic: k * G there, d / n - d and k / n - k chosen with
// masks, s = k + e d mod n with fixed limb loops.
int schnorr_sign(const uint8_t sk[32], const uint8_t msg[32], const uint8_t *aux_in, uint8_t sig[64]) {
    namespace k1 = chip::k1;
    {
        Bn d0;
        if (!parse_secret(sk, 32, d0)) return CHIP_ERR_SECP256K1;  // 0 < d < n (public check)
    }
    uint8_t aux[32];
    if (aux_in) std::memcpy(aux, aux_in, 32);
    else if (RAND_bytes(aux, 32) != 1) return CHIP_ERR_SECP256K1;
    uint8_t px[32], dd[32], t[32], rnd[32], rx[32], e32[32], o[65];
    if (!k1::to65(k1::mul_g(sk), o)) return CHIP_ERR_SECP256K1;
    std::memcpy(px, o + 1, 32);
    k1::Sc d = k1::sc_cond_neg(k1::sc_from_be(sk), o[64] & 1);  // the key with an even y
    k1::sc_to_be(d, dd);
    if (!tagged("BIP0340/aux", aux, 32, nullptr, 0, nullptr, 0, t)) return CHIP_ERR_SECP256K1;
    for (int i = 0; i < 32; ++i) t[i] ^= dd[i];
    if (!tagged("BIP0340/nonce", t, 32, px, 32, msg, 32, rnd)) return CHIP_ERR_SECP256K1;
    k1::Sc k = k1::sc_from_be(rnd);
    int st = CHIP_OK;
    if (k1::sc_is_zero(k)) st = CHIP_ERR_SECP256K1;  // probability ~2^-256
    uint8_t kb[32];
    k1::sc_to_be(k, kb);
    if (st == CHIP_OK && !k1::to65(k1::mul_g(kb), o)) st = CHIP_ERR_SECP256K1;
    if (st == CHIP_OK) {
        std::memcpy(rx, o + 1, 32);
        k = k1::sc_cond_neg(k, o[64] & 1);  // the nonce with an even y
        if (!tagged("BIP0340/challenge", rx, 32, px, 32, msg, 32, e32)) st = CHIP_ERR_SECP256K1;
    }
    if (st == CHIP_OK) {
        const k1::Sc s = k1::sc_add(k, k1::sc_mul(k1::sc_from_be(e32), d));  // s = (k + e d) mod n
        std::memcpy(sig, rx, 32);
        k1::sc_to_be(s, sig + 32);
    }
    k1::sc_clear(d);
    k1::sc_clear(k);
    OPENSSL_cleanse(dd, 32);
    OPENSSL_cleanse(t, 32);
    OPENSSL_cleanse(rnd, 32);
    OPENSSL_cleanse(kb, 32);
    return st;
}

// BIP-340 verify against the x-only key x32
int schnorr_verify_x(const uint8_t x32[32], const uint8_t msg[32], const uint8_t sig[64]) {
    Pt P;
    if (!lift_x(x32, P)) return CHIP_ERR_SECP256K1;
    Bn r(sig), s(sig + 32), e;
    if (BN_cmp(r.v, ctx().p) >= 0 || BN_cmp(s.v, order()) >= 0) return CHIP_ERR_SECP256K1;
    uint8_t e32[32], rx[32];
    if (!tagged("BIP0340/challenge", sig, 32, x32, 32, msg, 32, e32)) return CHIP_ERR_SECP256K1;
    BN_bin2bn(e32, 32, e.v);
    BN_mod(e.v, e.v, order(), ctx().bn);
    // R = s G - e P = s G + (n - e) P (public values); R must not be infinity,
    // must have an even y and x = r
    Bn ne;
    BN_sub(ne.v, order(), e.v);
    uint8_t sb[32], nb[32], xb[32], yb[32], o[65];
    bool even = false;
    if (!bn32(s.v, sb) || !bn32(ne.v, nb) || !xy(P.v, xb, &even)) return CHIP_ERR_SECP256K1;
    {
        Bn x, y;
        if (EC_POINT_get_affine_coordinates(ctx().g, P.v, x.v, y.v, ctx().bn) != 1 || !bn32(y.v, yb))
            return CHIP_ERR_SECP256K1;
    }
    namespace k1 = chip::k1;
    const k1::Pt R = k1::pt_add(k1::mul_g(sb), k1::mul(nb, k1::fe_from_be(xb), k1::fe_from_be(yb)));
    if (!k1::to65(R, o) || (o[64] & 1) || std::memcmp(o + 1, sig, 32) != 0) return CHIP_ERR_SECP256K1;
    (void)rx;
    return CHIP_OK;
}

void put_u32(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
uint32_t get_u32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

}  // namespace

extern "C" {

int chip_schnorr_sign(const uint8_t *sk, uint64_t sk_len, const uint8_t *msg, const uint8_t *aux, uint8_t *sig) {
    if (!sk || !msg || !sig) return CHIP_ERR_INVALID_ARG;
    if (sk_len != 32) return CHIP_ERR_SECP256K1;
    return schnorr_sign(sk, msg, aux, sig);
}

int chip_schnorr_verify(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *msg, const uint8_t *sig) {
    if (!pubkey || !msg || !sig) return CHIP_ERR_INVALID_ARG;
    uint8_t x[32];
    if (pubkey_len == 32) {  // x-only key
        std::memcpy(x, pubkey, 32);
    } else {
        Pt pt;
        bool even;
        if (!parse_public(pubkey, pubkey_len, pt) || !xy(pt.v, x, &even)) return CHIP_ERR_SECP256K1;
    }
    return schnorr_verify_x(x, msg, sig);
}

// Header::new (file.rs:263-289): message from the hash (32 bytes), pubkey
// from its bytes, the signature by the secret key, then decode_bao_hash.
int chip_header_new(const uint8_t *sk, uint64_t sk_len, const uint8_t *pk, uint64_t pk_len, const uint8_t *hash,
                    uint64_t hash_len, uint8_t format, uint8_t chunk_index, uint32_t encoded_len, uint32_t padding_len,
                    const uint8_t *metadata, const uint8_t *aux, chip_header *out) {
    if (!out || (!hash && hash_len) || (!pk && pk_len) || (!sk && sk_len)) return CHIP_ERR_INVALID_ARG;
    if (hash_len != 32) return CHIP_ERR_SECP256K1;  // Message::from_digest_slice
    Pt P;
    if (!parse_public(pk, pk_len, P)) return CHIP_ERR_SECP256K1;  // PublicKey::from_slice
    if (sk_len != 32) return CHIP_ERR_SECP256K1;                    // Keypair::from_seckey_slice
    chip_header h;
    std::memset(&h, 0, sizeof h);
    int st = schnorr_sign(sk, hash, aux, h.signature);
    if (st != CHIP_OK) return st;
    if (!compressed(P.v, h.pubkey)) return CHIP_ERR_SECP256K1;
    std::memcpy(h.hash, hash, 32);
    h.format = format;
    h.chunk_index = chunk_index;
    h.encoded_len = encoded_len;
    h.padding_len = padding_len;
    if (metadata) {
        std::memcpy(h.metadata, metadata, 8);
        h.has_metadata = 1;
    }
    *out = h;
    return CHIP_OK;
}

// Header::try_to_vec (file.rs:292-335)
int chip_header_to_bytes(const chip_header *h, uint8_t *out) {
    if (!h || !out) return CHIP_ERR_INVALID_ARG;
    uint8_t *p = out;
    std::memcpy(p, MAGIC, 12), p += 12;
    std::memcpy(p, h->pubkey, 33), p += 33;
    std::memcpy(p, h->hash, 32), p += 32;
    std::memcpy(p, h->signature, 64), p += 64;
    *p++ = h->format;
    *p++ = h->chunk_index;
    put_u32(p, h->encoded_len), p += 4;
    put_u32(p, h->padding_len), p += 4;
    if (h->has_metadata) std::memcpy(p, h->metadata, 8);
    else std::memset(p, 0, 8);
    p += 8;
    *p++ = 0;
    return (p - out) == CHIP_HEADER_LEN ? CHIP_OK : CHIP_ERR_INVALID_HEADER_LENGTH;
}

// Header::try_from(&[u8]) (file.rs:116-154, parse_bytes :345-392).  The
// reference unwraps the parser (a short slice panics, file.rs:126); here it is
// CHIP_ERR_INVALID_HEADER_LENGTH.  Metadata of all zeros reads as None.
int chip_header_parse(const uint8_t *b, uint64_t len, chip_header *out) {
    if (!out || (!b && len)) return CHIP_ERR_INVALID_ARG;
    if (len < CHIP_HEADER_LEN - 1) return CHIP_ERR_INVALID_HEADER_LENGTH;  // parse_bytes takes 159 bytes
    if (std::memcmp(b, MAGIC, 12) != 0) return CHIP_ERR_INVALID_MAGIC;
    chip_header h;
    std::memset(&h, 0, sizeof h);
    const uint8_t *p = b + 12;
    Pt P;
    if (!parse_public(p, 33, P)) return CHIP_ERR_SECP256K1;  // PublicKey::from_slice
    std::memcpy(h.pubkey, p, 33), p += 33;
    std::memcpy(h.hash, p, 32), p += 32;
    std::memcpy(h.signature, p, 64), p += 64;
    uint8_t x[32];
    bool even;
    if (!xy(P.v, x, &even)) return CHIP_ERR_SECP256K1;
    int st = schnorr_verify_x(x, h.hash, h.signature);  // file.rs:129-131
    if (st != CHIP_OK) return st;
    h.format = *p++;
    h.chunk_index = *p++;
    h.encoded_len = get_u32(p), p += 4;
    h.padding_len = get_u32(p), p += 4;
    std::memcpy(h.metadata, p, 8);
    for (int i = 0; i < 8; ++i) h.has_metadata |= p[i] != 0;
    *out = h;
    return CHIP_OK;
}

// file::encode (file.rs:409-440): the pubkey given, or derived from sk
// (compressed); encode(&pubkey, input, level); the header with chunk_index 0,
// encoded_len = output_len, padding_len; out = header || encoded.
int chip_file_encode(const uint8_t *sk, uint64_t sk_len, const uint8_t *pk, uint64_t pk_len, const uint8_t *in,
                     uint64_t n, uint8_t level, const uint8_t *metadata, const chip_ecies_inject *inject,
                     const uint8_t *aux, uint8_t *out, uint64_t cap, uint64_t *out_len, chip_encode_info *info) {
    if (!out_len || (!in && n) || (!sk && sk_len) || (!pk && pk_len)) return CHIP_ERR_INVALID_ARG;
    uint8_t pub[33];
    if (pk && pk_len) {
        Pt P;
        if (!parse_public(pk, pk_len, P) || !compressed(P.v, pub)) return CHIP_ERR_SECP256K1;
    } else {
        Bn d;
        bool even = false;
        if (!parse_secret(sk, sk_len, d) || !mul_g_xy(d.v, pub + 1, &even)) return CHIP_ERR_SECP256K1;
        pub[0] = even ? 0x02 : 0x03;
    }
    uint64_t max = chip_encode_max_len(n);
    if (!out || cap < CHIP_HEADER_LEN) {
        *out_len = CHIP_HEADER_LEN + max;
        return CHIP_ERR_BUFFER_TOO_SMALL;
    }
    uint8_t hash[32];
    chip_encode_info inf;
    uint64_t blen = 0;
    int st = chip_encode(level, pub, 33, inject, in, n, out + CHIP_HEADER_LEN, cap - CHIP_HEADER_LEN, &blen, hash, &inf);
    if (st == CHIP_ERR_BUFFER_TOO_SMALL) {
        *out_len = CHIP_HEADER_LEN + blen;
        return st;
    }
    if (st != CHIP_OK) return st;
    chip_header h;
    st = chip_header_new(sk, sk_len, pub, 33, hash, 32, level, 0, inf.output_len, inf.padding_len, metadata, aux, &h);
    if (st != CHIP_OK) return st;
    st = chip_header_to_bytes(&h, out);
    if (st != CHIP_OK) return st;
    *out_len = CHIP_HEADER_LEN + blen;
    if (info) *info = inf;
    return CHIP_OK;
}

// file::decode (file.rs:395-407): split at the header, parse and verify it,
// decode(sk, hash, body, padding, format).
int chip_file_decode(const uint8_t *sk, uint64_t sk_len, const uint8_t *in, uint64_t n, chip_header *hdr,
                     uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (!out_len || (!in && n)) return CHIP_ERR_INVALID_ARG;
    if (n < CHIP_HEADER_LEN) return CHIP_ERR_INVALID_HEADER_LENGTH;  // split_at panics in the reference
    chip_header h;
    int st = chip_header_parse(in, CHIP_HEADER_LEN, &h);
    if (st != CHIP_OK) return st;
    if (hdr) *hdr = h;
    return chip_decode(sk, sk_len, h.hash, 32, in + CHIP_HEADER_LEN, n - CHIP_HEADER_LEN, h.padding_len, h.format, out,
                       cap, out_len);
}

}  // extern "C"
