// secp256k1_host.hpp — constant-time secp256k1 scalar multiplication for the
// host ECIES stage (ecies 0.2 over libsecp256k1: encoding.rs:31-36,
// decoding.rs:62-69).
//
// OpenSSL has no dedicated secp256k1 code: its generic prime-field ladder set
// most of the latency of a small level-15 encode() (~450 us on the GPU box,
// DESIGN.md §6; ECIES does two scalar multiplications per encrypt and one
// per decrypt).  This is a small dedicated implementation (on the GPU box's
// CPU: k * P 34 us, k * G 15 us, tools/secp_field_check, r10h):
//
//  * field elements: five 52-bit limbs with lazy reduction (magnitudes, see
//    Fe below), products through unsigned __int128, 2^256 = 2^32 + 977
//    (mod p); fe_norm gives the canonical value for output and zero tests.
//    Every function runs the same instructions whatever the values (no
//    branches or table indices on them); fe_inv is a fixed addition chain;
//  * points: projective (X : Y : Z) with the complete formulas of Renes,
//    Costello and Batina (EUROCRYPT 2016), Algorithms 7 (addition) and 9
//    (doubling) for a = 0, b3 = 21.  They have no exceptional cases, so the
//    point at infinity and equal operands need no branches;
//  * k * P: k split with the endomorphism (GLV: k = k1 + k2 lambda, |k_i| <
//    2^128, negative halves as n - k_i with the point's y negated by masks),
//    33 joint 4-bit windows: 132 doublings and 66 additions; each window's
//    multiple is read by scanning the whole 16-entry table with masks;
//  * k * G: a precomputed table of i * 16^j * G (64 x 16 points, built once
//    per process), 64 additions and no doublings, the same masked scans;
//  * scalars mod n (BIP-340 signing): fixed limb loops, results chosen with
//    masks.
//
// Scalars are 32-byte big-endian with 0 < k < n (the caller checks, as
// libsecp256k1's SecretKey::parse).  tests/test_host_stages.py and
// tests/test_secp_field.py compare k * G, the field and point arithmetic and
// the ECIES envelopes (k * P inside) with the C and Python oracles'
// independent secp256k1 code on edge-case and random scalars;
// tests/test_constant_time.py (tests/dudect_ct.cpp) gives the timing
// evidence: Welch's t over cycle counts, fixed vs random secret, 10^5
// samples per class, |t| < 4.5 for k * P, k * G, fe_inv, the signing scalars,
// BIP-340 signing end to end and the AES-GCM tag check.
#pragma once

#include <immintrin.h>

#include <cstdint>
#include <cstring>

namespace chip {
namespace k1 {

typedef unsigned __int128 u128;

// Field elements: five 52-bit limbs, value = sum v[i] 2^(52 i), reduced
// lazily.  "Magnitude" m bounds the limbs by about m 2^52 (v[4]: m 2^48).
// fe_mul / fe_sqr / fe_sub / fe_mul21 / fe_weak return magnitude 1 (limbs
// < 2^52 + 2^34); fe_add adds magnitudes and is the only function that
// grows them.  fe_mul and fe_sqr accept magnitude <= 8 (limbs < 2^56: five
// 112-bit products per column fit 128 bits), fe_sub a subtrahend of
// magnitude <= 8.  fe_norm gives the unique representative in [0, p) for
// output and zero tests.  No branches or table indices on the values.
struct Fe {
    uint64_t v[5];
};

constexpr uint64_t M52 = 0xFFFFFFFFFFFFFull, M48 = 0xFFFFFFFFFFFFull;
constexpr uint64_t RC = 0x1000003D1ull;      // 2^256 mod p
constexpr uint64_t R260 = 0x1000003D10ull;   // 2^260 mod p (limb 5 folds onto limb 0)
// 16 p, limb by limb (each limb >= 16 x a magnitude-1 limb bound / 2): a - b = a + 16p - b
constexpr uint64_t P16_0 = 0xFFFFEFFFFFC2Full * 16, P16_1 = M52 * 16, P16_4 = M48 * 16;

// carry the limbs down to 52 bits, the bits above 2^256 folded with RC
inline Fe fe_weak(const Fe &a) {
    uint64_t t0 = a.v[0], t1 = a.v[1], t2 = a.v[2], t3 = a.v[3], t4 = a.v[4];
    const uint64_t x = t4 >> 48;
    t4 &= M48;
    t0 += x * RC;
    t1 += t0 >> 52, t0 &= M52;
    t2 += t1 >> 52, t1 &= M52;
    t3 += t2 >> 52, t2 &= M52;
    t4 += t3 >> 52, t3 &= M52;
    return Fe{{t0, t1, t2, t3, t4}};
}

// [0, p): two carry passes (value < 2^256), then p subtracted once if value >= p
inline Fe fe_norm(const Fe &a) {
    Fe r = fe_weak(fe_weak(a));
    // value + (2^256 - p) reaches 2^256 iff value >= p
    uint64_t u0 = r.v[0] + RC, u1 = r.v[1] + (u0 >> 52), u2, u3, u4;
    u0 &= M52;
    u2 = r.v[2] + (u1 >> 52), u1 &= M52;
    u3 = r.v[3] + (u2 >> 52), u2 &= M52;
    u4 = r.v[4] + (u3 >> 52), u3 &= M52;
    const uint64_t ge = 0 - (u4 >> 48);  // all ones: value >= p, take the sum mod 2^256
    u4 &= M48;
    return Fe{{(u0 & ge) | (r.v[0] & ~ge), (u1 & ge) | (r.v[1] & ~ge), (u2 & ge) | (r.v[2] & ~ge),
               (u3 & ge) | (r.v[3] & ~ge), (u4 & ge) | (r.v[4] & ~ge)}};
}

// the ten columns of a product (52 bits, t[5] < 2^63, t[9] the top carry)
// folded to magnitude 1: t[5 + k] 2^(260 + 52 k) = t[5 + k] R260 2^(52 k)
inline Fe fe_fold(const uint64_t t[10]) {
    u128 c = (u128)t[5] * R260 + t[0];
    const uint64_t r0 = (uint64_t)c & M52;
    c = (c >> 52) + (u128)t[6] * R260 + t[1];
    const uint64_t r1 = (uint64_t)c & M52;
    c = (c >> 52) + (u128)t[7] * R260 + t[2];
    const uint64_t r2 = (uint64_t)c & M52;
    c = (c >> 52) + (u128)t[8] * R260 + t[3];
    const uint64_t r3 = (uint64_t)c & M52;
    c = (c >> 52) + (u128)t[9] * R260 + t[4];
    const uint64_t r4 = (uint64_t)c & M48;
    c = (u128)(uint64_t)(c >> 48) * RC + r0;  // the bits above 2^256 (< 2^50)
    return Fe{{(uint64_t)c & M52, r1 + (uint64_t)(c >> 52), r2, r3, r4}};
}

// The column sums are independent of each other (balanced trees of
// products); the 52-bit carries run through columns 0-4 and 5-8 as two
// chains side by side, column 4's carry joining t[5] (< 2^63) at the end.
inline Fe fe_cols(u128 c0, u128 c1, u128 c2, u128 c3, u128 c4, u128 c5, u128 c6, u128 c7, u128 c8) {
    uint64_t t[10];
    t[0] = (uint64_t)c0 & M52;
    c1 += c0 >> 52;
    t[5] = (uint64_t)c5 & M52;
    c6 += c5 >> 52;
    t[1] = (uint64_t)c1 & M52;
    c2 += c1 >> 52;
    t[6] = (uint64_t)c6 & M52;
    c7 += c6 >> 52;
    t[2] = (uint64_t)c2 & M52;
    c3 += c2 >> 52;
    t[7] = (uint64_t)c7 & M52;
    c8 += c7 >> 52;
    t[3] = (uint64_t)c3 & M52;
    c4 += c3 >> 52;
    t[8] = (uint64_t)c8 & M52;
    t[9] = (uint64_t)(c8 >> 52);
    t[4] = (uint64_t)c4 & M52;
    t[5] += (uint64_t)(c4 >> 52);
    return fe_fold(t);
}

inline Fe fe_mul(const Fe &a, const Fe &b) {
    const uint64_t *x = a.v, *y = b.v;
    auto m = [](uint64_t u, uint64_t v) { return (u128)u * v; };
    return fe_cols(m(x[0], y[0]), m(x[0], y[1]) + m(x[1], y[0]), (m(x[0], y[2]) + m(x[1], y[1])) + m(x[2], y[0]),
                   (m(x[0], y[3]) + m(x[1], y[2])) + (m(x[2], y[1]) + m(x[3], y[0])),
                   (m(x[0], y[4]) + m(x[1], y[3])) + (m(x[2], y[2]) + m(x[3], y[1])) + m(x[4], y[0]),
                   (m(x[1], y[4]) + m(x[2], y[3])) + (m(x[3], y[2]) + m(x[4], y[1])),
                   (m(x[2], y[4]) + m(x[3], y[3])) + m(x[4], y[2]), m(x[3], y[4]) + m(x[4], y[3]), m(x[4], y[4]));
}

inline Fe fe_sqr(const Fe &a) {  // 15 products: the cross terms once, doubled
    const uint64_t *x = a.v;
    const uint64_t d0 = 2 * x[0], d1 = 2 * x[1], d2 = 2 * x[2], d3 = 2 * x[3];
    auto m = [](uint64_t u, uint64_t v) { return (u128)u * v; };
    return fe_cols(m(x[0], x[0]), m(d0, x[1]), m(d0, x[2]) + m(x[1], x[1]), m(d0, x[3]) + m(d1, x[2]),
                   (m(d0, x[4]) + m(d1, x[3])) + m(x[2], x[2]), m(d1, x[4]) + m(d2, x[3]),
                   m(d2, x[4]) + m(x[3], x[3]), m(d3, x[4]), m(x[4], x[4]));
}

inline Fe fe_add(const Fe &a, const Fe &b) {  // magnitudes add
    return Fe{{a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3], a.v[4] + b.v[4]}};
}

inline Fe fe_sub(const Fe &a, const Fe &b) {  // a + 16p - b (b of magnitude <= 8)
    return fe_weak(Fe{{a.v[0] + P16_0 - b.v[0], a.v[1] + P16_1 - b.v[1], a.v[2] + P16_1 - b.v[2],
                       a.v[3] + P16_1 - b.v[3], a.v[4] + P16_4 - b.v[4]}});
}

inline Fe fe_mul21(const Fe &a) {  // b3 = 3 * 7
    return fe_weak(Fe{{a.v[0] * 21, a.v[1] * 21, a.v[2] * 21, a.v[3] * 21, a.v[4] * 21}});
}

inline Fe fe_sqr_n(Fe a, int n) {
    for (int i = 0; i < n; ++i) a = fe_sqr(a);
    return a;
}

// a^(p-2) (a != 0) by the addition chain over the blocks of ones of p - 2
// (lengths 1, 2, 22 and 223): 255 squarings and 15 multiplications
inline Fe fe_inv(const Fe &a) {
    const Fe x2 = fe_mul(fe_sqr(a), a);
    const Fe x3 = fe_mul(fe_sqr(x2), a);
    const Fe x6 = fe_mul(fe_sqr_n(x3, 3), x3);
    const Fe x9 = fe_mul(fe_sqr_n(x6, 3), x3);
    const Fe x11 = fe_mul(fe_sqr_n(x9, 2), x2);
    const Fe x22 = fe_mul(fe_sqr_n(x11, 11), x11);
    const Fe x44 = fe_mul(fe_sqr_n(x22, 22), x22);
    const Fe x88 = fe_mul(fe_sqr_n(x44, 44), x44);
    const Fe x176 = fe_mul(fe_sqr_n(x88, 88), x88);
    const Fe x220 = fe_mul(fe_sqr_n(x176, 44), x44);
    const Fe x223 = fe_mul(fe_sqr_n(x220, 3), x3);
    Fe t = fe_mul(fe_sqr_n(x223, 23), x22);
    t = fe_mul(fe_sqr_n(t, 5), a);
    t = fe_mul(fe_sqr_n(t, 3), x2);
    return fe_mul(fe_sqr_n(t, 2), a);
}

// a^((p+1)/4), a square root of a when a is a square (p = 3 mod 4; the
// caller checks r^2 == a).  The blocks of ones of (p+1)/4 are 223, 22 and 2
// bits long: 253 squarings and 13 multiplications.
inline Fe fe_sqrt_cand(const Fe &a) {
    const Fe x2 = fe_mul(fe_sqr(a), a);
    const Fe x3 = fe_mul(fe_sqr(x2), a);
    const Fe x6 = fe_mul(fe_sqr_n(x3, 3), x3);
    const Fe x9 = fe_mul(fe_sqr_n(x6, 3), x3);
    const Fe x11 = fe_mul(fe_sqr_n(x9, 2), x2);
    const Fe x22 = fe_mul(fe_sqr_n(x11, 11), x11);
    const Fe x44 = fe_mul(fe_sqr_n(x22, 22), x22);
    const Fe x88 = fe_mul(fe_sqr_n(x44, 44), x44);
    const Fe x176 = fe_mul(fe_sqr_n(x88, 88), x88);
    const Fe x220 = fe_mul(fe_sqr_n(x176, 44), x44);
    const Fe x223 = fe_mul(fe_sqr_n(x220, 3), x3);
    Fe t = fe_mul(fe_sqr_n(x223, 23), x22);
    t = fe_mul(fe_sqr_n(t, 6), x2);
    return fe_sqr_n(t, 2);
}

// 32 big-endian bytes (< 2^256) -> magnitude 1
inline Fe fe_from_be(const uint8_t b[32]) {
    uint64_t w[4];
    for (int i = 0; i < 4; ++i) {
        uint64_t x = 0;
        for (int j = 0; j < 8; ++j) x = (x << 8) | b[(3 - i) * 8 + j];
        w[i] = x;
    }
    return Fe{{w[0] & M52, ((w[0] >> 52) | (w[1] << 12)) & M52, ((w[1] >> 40) | (w[2] << 24)) & M52,
               ((w[2] >> 28) | (w[3] << 36)) & M52, w[3] >> 16}};
}

inline void fe_to_be(const Fe &f, uint8_t b[32]) {
    const Fe n = fe_norm(f);
    const uint64_t w[4] = {n.v[0] | (n.v[1] << 52), (n.v[1] >> 12) | (n.v[2] << 40), (n.v[2] >> 24) | (n.v[3] << 28),
                           (n.v[3] >> 36) | (n.v[4] << 16)};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(w[i] >> (56 - 8 * j));
}

inline bool fe_is_zero(const Fe &f) {
    const Fe n = fe_norm(f);
    return (n.v[0] | n.v[1] | n.v[2] | n.v[3] | n.v[4]) == 0;
}

// A compressed point (0x02 / 0x03 || x, 33 bytes) -> affine x, y, as
// libsecp256k1's PublicKey::parse and OpenSSL's oct2point accept it: false
// unless x < p and x^3 + 7 is a square; y the root of the tag's parity.
constexpr uint8_t P_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                              0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                              0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xFF, 0xFF, 0xFC, 0x2F};

inline bool decompress(const uint8_t in[33], Fe &x, Fe &y) {
    if ((in[0] != 0x02 && in[0] != 0x03) || std::memcmp(in + 1, P_BE, 32) >= 0) return false;
    x = fe_from_be(in + 1);
    const Fe y2 = fe_add(fe_mul(fe_sqr(x), x), Fe{{7, 0, 0, 0, 0}});
    Fe r = fe_sqrt_cand(y2);
    if (!fe_is_zero(fe_sub(fe_sqr(r), y2))) return false;
    r = fe_norm(r);
    if ((r.v[0] & 1) != (uint64_t)(in[0] & 1)) r = fe_norm(fe_sub(Fe{{0, 0, 0, 0, 0}}, r));
    y = r;
    return true;
}

// An uncompressed point (0x04 || x || y, 65 bytes), as libsecp256k1's
// PublicKey::parse and OpenSSL's oct2point accept that form: false unless
// x, y < p and y^2 = x^3 + 7.
inline bool parse_full(const uint8_t in[65], Fe &x, Fe &y) {
    if (in[0] != 0x04 || std::memcmp(in + 1, P_BE, 32) >= 0 || std::memcmp(in + 33, P_BE, 32) >= 0) return false;
    x = fe_from_be(in + 1);
    y = fe_from_be(in + 33);
    return fe_is_zero(fe_sub(fe_sqr(y), fe_add(fe_mul(fe_sqr(x), x), Fe{{7, 0, 0, 0, 0}})));
}

struct Pt {
    Fe x, y, z;  // projective; infinity = (0 : 1 : 0)
};

inline Pt pt_inf() { return Pt{{{0, 0, 0, 0, 0}}, {{1, 0, 0, 0, 0}}, {{0, 0, 0, 0, 0}}}; }

// Renes-Costello-Batina Algorithm 7 (a = 0): complete addition
inline Pt pt_add(const Pt &p, const Pt &q) {
    Fe t0 = fe_mul(p.x, q.x), t1 = fe_mul(p.y, q.y), t2 = fe_mul(p.z, q.z);
    Fe t3 = fe_add(p.x, p.y), t4 = fe_add(q.x, q.y);
    t3 = fe_mul(t3, t4);
    t4 = fe_add(t0, t1);
    t3 = fe_sub(t3, t4);
    t4 = fe_add(p.y, p.z);
    Fe x3 = fe_add(q.y, q.z);
    t4 = fe_mul(t4, x3);
    x3 = fe_add(t1, t2);
    t4 = fe_sub(t4, x3);
    x3 = fe_add(p.x, p.z);
    Fe y3 = fe_add(q.x, q.z);
    x3 = fe_mul(x3, y3);
    y3 = fe_add(t0, t2);
    y3 = fe_sub(x3, y3);
    x3 = fe_add(t0, t0);
    t0 = fe_add(x3, t0);
    t2 = fe_mul21(t2);
    Fe z3 = fe_add(t1, t2);
    t1 = fe_sub(t1, t2);
    y3 = fe_mul21(y3);
    x3 = fe_mul(t4, y3);
    t2 = fe_mul(t3, t1);
    x3 = fe_sub(t2, x3);
    y3 = fe_mul(y3, t0);
    t1 = fe_mul(t1, z3);
    y3 = fe_add(t1, y3);
    t0 = fe_mul(t0, t3);
    z3 = fe_mul(z3, t4);
    z3 = fe_add(z3, t0);
    return Pt{x3, y3, z3};
}

// Renes-Costello-Batina Algorithm 9 (a = 0): complete doubling
inline Pt pt_dbl(const Pt &p) {
    Fe t0 = fe_sqr(p.y);
    Fe z3 = fe_add(t0, t0);
    z3 = fe_add(z3, z3);
    z3 = fe_add(z3, z3);
    Fe t1 = fe_mul(p.y, p.z), t2 = fe_sqr(p.z);
    t2 = fe_mul21(t2);
    Fe x3 = fe_mul(t2, z3), y3 = fe_add(t0, t2);
    z3 = fe_mul(t1, z3);
    t1 = fe_add(t2, t2);
    t2 = fe_add(t1, t2);
    t0 = fe_sub(t0, t2);
    y3 = fe_mul(t0, y3);
    y3 = fe_add(x3, y3);
    t1 = fe_mul(p.x, p.y);
    x3 = fe_mul(t0, t1);
    x3 = fe_add(x3, x3);
    return Pt{x3, y3, z3};
}

// table[w] without a data-dependent index: every entry read, one kept
inline Pt pt_select(const Pt (&table)[16], uint32_t w) {
    Pt r;
    std::memset(&r, 0, sizeof r);
    for (uint32_t i = 0; i < 16; ++i) {
        const uint64_t m = 0 - (((uint64_t)(i ^ w) - 1) >> 63);  // all ones iff i == w
        const uint64_t *s = reinterpret_cast<const uint64_t *>(&table[i]);
        uint64_t *d = reinterpret_cast<uint64_t *>(&r);
        for (size_t k = 0; k < sizeof(Pt) / 8; ++k) d[k] |= s[k] & m;
    }
    return r;
}

inline uint32_t nibble(const uint8_t k[32], int j) {  // j-th 4-bit window from the least significant end
    const uint8_t b = k[31 - j / 2];
    return (j & 1) ? (b >> 4) : (b & 15u);
}

inline const Fe &gx() {
    static const uint8_t b[32] = {0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62,
                                  0x95, 0xCE, 0x87, 0x0B, 0x07, 0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE,
                                  0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
    static const Fe f = fe_from_be(b);
    return f;
}

inline const Fe &gy() {
    static const uint8_t b[32] = {0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB,
                                  0xFC, 0x0E, 0x11, 0x08, 0xA8, 0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85,
                                  0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};
    static const Fe f = fe_from_be(b);
    return f;
}

// Fixed-base comb: i * 16^j * P for j < 64, i < 16 (~0.3 ms to build); k * P
// is then 64 complete additions of full-table-scan picks, no doublings.  For
// G (built on first use) and for a receiver key seen again (host_stages.cpp).
struct CombTable {
    Pt t[64][16];
    CombTable(const Fe &x, const Fe &y) {
        Pt base{x, y, {{1, 0, 0, 0, 0}}};
        for (int j = 0; j < 64; ++j) {
            t[j][0] = pt_inf();
            t[j][1] = base;
            for (int i = 2; i < 16; ++i) t[j][i] = pt_add(t[j][i - 1], base);
            base = pt_dbl(pt_dbl(pt_dbl(pt_dbl(base))));
        }
    }
};

inline const CombTable &gtable() {
    static const CombTable *g = new CombTable(gx(), gy());  // never destroyed (used from host-stage threads)
    return *g;
}

// k * P from P's comb table, 0 <= k < 2^256 (every step the same for every k)
inline Pt mul_comb(const CombTable &tb, const uint8_t k[32]) {
    Pt r = pt_inf();
    for (int j = 0; j < 64; ++j) r = pt_add(r, pt_select(tb.t[j], nibble(k, j)));
    return r;
}

inline Pt mul_g(const uint8_t k[32]) { return mul_comb(gtable(), k); }

// affine (x, y) of a point other than infinity, as 0x04 || x || y
inline bool to65(const Pt &p, uint8_t out[65]) {
    if (fe_is_zero(p.z)) return false;  // infinity (public: a failed operation)
    const Fe zi = fe_inv(p.z);
    out[0] = 0x04;
    fe_to_be(fe_mul(p.x, zi), out + 1);
    fe_to_be(fe_mul(p.y, zi), out + 33);
    return true;
}

// to65 of two points with one inversion (1 / z1 = z2 / (z1 z2), and so on)
inline bool to65_pair(const Pt &p, const Pt &q, uint8_t op[65], uint8_t oq[65]) {
    if (fe_is_zero(p.z) || fe_is_zero(q.z)) return false;
    const Fe i = fe_inv(fe_mul(p.z, q.z));
    const Fe pi = fe_mul(i, q.z), qi = fe_mul(i, p.z);
    op[0] = oq[0] = 0x04;
    fe_to_be(fe_mul(p.x, pi), op + 1);
    fe_to_be(fe_mul(p.y, pi), op + 33);
    fe_to_be(fe_mul(q.x, qi), oq + 1);
    fe_to_be(fe_mul(q.y, qi), oq + 33);
    return true;
}

// ---- scalars mod n (BIP-340 signing: s = k + e d, d or n - d) ------------
// Fixed limb counts and loops, results chosen with masks: the same
// instructions run whatever the key or nonce (OpenSSL's BIGNUM arithmetic
// branches on the values).  Reduction mod n as libsecp256k1's: with
// C = 2^256 - n (129 bits), x = hi 2^256 + lo = hi C + lo (mod n), folded
// three times, then one conditional subtraction.
struct Sc {
    uint64_t v[4];  // little-endian limbs, < n
};

constexpr uint64_t N0 = 0xBFD25E8CD0364141ull, N1 = 0xBAAEDCE6AF48A03Bull, N2 = 0xFFFFFFFFFFFFFFFEull,
                   N3 = 0xFFFFFFFFFFFFFFFFull;
constexpr uint64_t NC[3] = {0x402DA1732FC9BEBFull, 0x4551231950B75FC4ull, 1ull};  // 2^256 - n

// out += a * b (AL x BL limbs); carries run to the end of out (OL limbs)
template <int AL, int BL, int OL>
inline void sc_mac(uint64_t (&out)[OL], const uint64_t *a, const uint64_t *b) {
    for (int i = 0; i < AL; ++i) {
        uint64_t carry = 0;
        for (int j = 0; j < BL; ++j) {
            const u128 acc = (u128)a[i] * b[j] + out[i + j] + carry;
            out[i + j] = (uint64_t)acc;
            carry = (uint64_t)(acc >> 64);
        }
        for (int k = i + BL; k < OL; ++k) {
            const u128 acc = (u128)out[k] + carry;
            out[k] = (uint64_t)acc;
            carry = (uint64_t)(acc >> 64);
        }
    }
}

// x (5 limbs, < 2n) -> x mod n
inline Sc sc_reduce_once(const uint64_t (&x)[5]) {
    unsigned long long s0, s1, s2, s3, s4;
    unsigned char b = _subborrow_u64(0, x[0], N0, &s0);
    b = _subborrow_u64(b, x[1], N1, &s1);
    b = _subborrow_u64(b, x[2], N2, &s2);
    b = _subborrow_u64(b, x[3], N3, &s3);
    b = _subborrow_u64(b, x[4], 0, &s4);
    const uint64_t keep = 0 - (uint64_t)b;  // all ones: x < n
    Sc r;
    r.v[0] = (x[0] & keep) | (s0 & ~keep);
    r.v[1] = (x[1] & keep) | (s1 & ~keep);
    r.v[2] = (x[2] & keep) | (s2 & ~keep);
    r.v[3] = (x[3] & keep) | (s3 & ~keep);
    return r;
}

// 32 big-endian bytes (any value < 2^256 < 2n) -> value mod n
inline Sc sc_from_be(const uint8_t b[32]) {
    uint64_t x[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 32; ++i) x[3 - i / 8] |= (uint64_t)b[i] << (8 * (7 - i % 8));
    return sc_reduce_once(x);
}

inline void sc_to_be(const Sc &a, uint8_t b[32]) {
    for (int i = 0; i < 32; ++i) b[i] = (uint8_t)(a.v[3 - i / 8] >> (8 * (7 - i % 8)));
}

inline Sc sc_add(const Sc &a, const Sc &b) {
    uint64_t x[5];
    unsigned long long t;
    unsigned char c = _addcarry_u64(0, a.v[0], b.v[0], &t);
    x[0] = t;
    c = _addcarry_u64(c, a.v[1], b.v[1], &t);
    x[1] = t;
    c = _addcarry_u64(c, a.v[2], b.v[2], &t);
    x[2] = t;
    c = _addcarry_u64(c, a.v[3], b.v[3], &t);
    x[3] = t;
    x[4] = c;
    return sc_reduce_once(x);
}

// neg ? n - a : a, for 0 < a < n
inline Sc sc_cond_neg(const Sc &a, bool neg) {
    unsigned long long m0, m1, m2, m3;
    unsigned char b = _subborrow_u64(0, N0, a.v[0], &m0);
    b = _subborrow_u64(b, N1, a.v[1], &m1);
    b = _subborrow_u64(b, N2, a.v[2], &m2);
    (void)_subborrow_u64(b, N3, a.v[3], &m3);
    const uint64_t sel = 0 - (uint64_t)neg;
    Sc r;
    r.v[0] = (m0 & sel) | (a.v[0] & ~sel);
    r.v[1] = (m1 & sel) | (a.v[1] & ~sel);
    r.v[2] = (m2 & sel) | (a.v[2] & ~sel);
    r.v[3] = (m3 & sel) | (a.v[3] & ~sel);
    return r;
}

inline Sc sc_mul(const Sc &a, const Sc &b) {
    uint64_t l[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    sc_mac<4, 4, 8>(l, a.v, b.v);                               // < n^2 < 2^512
    uint64_t m[7] = {l[0], l[1], l[2], l[3], 0, 0, 0};
    sc_mac<4, 3, 7>(m, l + 4, NC);                              // < 2^256 + 2^385
    uint64_t p[5] = {m[0], m[1], m[2], m[3], 0};
    sc_mac<3, 3, 5>(p, m + 4, NC);                              // m >> 256 < 2^130: < 2^260
    uint64_t r[5] = {p[0], p[1], p[2], p[3], 0};
    sc_mac<1, 3, 5>(r, p + 4, NC);                              // p >> 256 < 2^4: < 2^256 + 2^133 < 2n
    return sc_reduce_once(r);
}

inline bool sc_is_zero(const Sc &a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }

inline void sc_clear(Sc &a) {
    volatile uint64_t *p = a.v;
    for (int i = 0; i < 4; ++i) p[i] = 0;
}

// ---- k * P with the endomorphism (GLV) ------------------------------------
// lambda (x, y) = (beta x, y) for the cube roots of unity lambda mod n and
// beta mod p.  k = k1 + k2 lambda (mod n) with |k1|, |k2| < 2^128 (the
// lattice split: c1 = round(b2 k / n), c2 = round(-b1 k / n) through
// g = round(2^384 b / n); k2 = c1 (-b1) + c2 (-b2), k1 = k - k2 lambda), so
// k P = k1 P + k2 (lambda P) takes 128 doublings instead of 256.  Negative
// halves are taken as n - k_i with the point's y negated.  Every step is
// the same for every k (masks, full table scans, fixed loop counts).
constexpr Sc GLV_G1 = {{0xe893209a45dbb031ull, 0x3daa8a1471e8ca7full, 0xe86c90e49284eb15ull, 0x3086d221a7d46bcdull}};
constexpr Sc GLV_G2 = {{0x1571b4ae8ac47f71ull, 0x221208ac9df506c6ull, 0x6f547fa90abfe4c4ull, 0xe4437ed6010e8828ull}};
constexpr Sc GLV_MB1 = {{0x6f547fa90abfe4c3ull, 0xe4437ed6010e8828ull, 0, 0}};  // -b1
constexpr Sc GLV_MB2 = {{0xd765cda83db1562cull, 0x8a280ac50774346dull, 0xfffffffffffffffeull,
                         0xffffffffffffffffull}};  // -b2 mod n
constexpr Sc GLV_MLAM = {{0xe0cfc810b51283cfull, 0xa880b9fc8ec739c2ull, 0x5ad9e3fd77ed9ba4ull,
                          0xac9c52b33fa3cf1full}};  // -lambda mod n

inline const Fe &glv_beta() {
    static const uint8_t b[32] = {0x7a, 0xe9, 0x6a, 0x2b, 0x65, 0x7c, 0x07, 0x10, 0x6e, 0x64, 0x47,
                                  0x9e, 0xac, 0x34, 0x34, 0xe9, 0x9c, 0xf0, 0x49, 0x75, 0x12, 0xf5,
                                  0x89, 0x95, 0xc1, 0x39, 0x6c, 0x28, 0x71, 0x95, 0x01, 0xee};
    static const Fe f = fe_from_be(b);
    return f;
}

// round(k g / 2^384) (< 2^128)
inline Sc sc_mulshift384(const Sc &k, const Sc &g) {
    uint64_t l[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    sc_mac<4, 4, 8>(l, k.v, g.v);
    unsigned long long lo, hi;
    const unsigned char c = _addcarry_u64(0, l[6], l[5] >> 63, &lo);
    (void)_addcarry_u64(c, l[7], 0, &hi);
    return Sc{{lo, hi, 0, 0}};
}

// all ones iff a > (n - 1) / 2
inline uint64_t sc_high_mask(const Sc &a) {
    constexpr uint64_t H0 = 0xDFE92F46681B20A0ull, H1 = 0x5D576E7357A4501Dull, H2 = 0xFFFFFFFFFFFFFFFFull,
                       H3 = 0x7FFFFFFFFFFFFFFFull;
    unsigned long long t;
    unsigned char b = _subborrow_u64(0, H0, a.v[0], &t);
    b = _subborrow_u64(b, H1, a.v[1], &t);
    b = _subborrow_u64(b, H2, a.v[2], &t);
    b = _subborrow_u64(b, H3, a.v[3], &t);
    return 0 - (uint64_t)b;
}

inline Fe fe_cmov(const Fe &a, const Fe &b, uint64_t m) {  // m all ones: b, else a
    Fe r;
    for (int i = 0; i < 5; ++i) r.v[i] = (a.v[i] & ~m) | (b.v[i] & m);
    return r;
}

inline uint32_t sc_nibble(const Sc &a, int j) { return (uint32_t)(a.v[j >> 4] >> (4 * (j & 15))) & 15u; }

// k * P for an affine point P = (x, y), 0 < k < n
inline Pt mul(const uint8_t k[32], const Fe &x, const Fe &y) {
    const Sc s = sc_from_be(k);
    const Sc c1 = sc_mulshift384(s, GLV_G1), c2 = sc_mulshift384(s, GLV_G2);
    const Sc k2 = sc_add(sc_mul(c1, GLV_MB1), sc_mul(c2, GLV_MB2));
    const Sc k1 = sc_add(s, sc_mul(k2, GLV_MLAM));
    const uint64_t n1 = sc_high_mask(k1), n2 = sc_high_mask(k2);
    const Sc a1 = sc_cond_neg(k1, n1 != 0), a2 = sc_cond_neg(k2, n2 != 0);
    const Fe zero = {{0, 0, 0, 0, 0}};
    // T1[i] = i (+-P), T2[i] = lambda T1[i] with y negated again when the signs differ
    Pt t1[16], t2[16];
    t1[0] = pt_inf();
    t1[1] = Pt{x, fe_cmov(y, fe_sub(zero, y), n1), {{1, 0, 0, 0, 0}}};
    for (int i = 2; i < 16; ++i) t1[i] = pt_add(t1[i - 1], t1[1]);
    const uint64_t flip = n1 ^ n2;
    for (int i = 0; i < 16; ++i)
        t2[i] = Pt{fe_mul(t1[i].x, glv_beta()), fe_cmov(t1[i].y, fe_sub(zero, t1[i].y), flip), t1[i].z};
    Pt r = pt_inf();
    for (int j = 32; j >= 0; --j) {  // 33 windows: 132 bits, |k_i| < 2^128
        r = pt_dbl(pt_dbl(pt_dbl(pt_dbl(r))));
        r = pt_add(r, pt_select(t1, sc_nibble(a1, j)));
        r = pt_add(r, pt_select(t2, sc_nibble(a2, j)));
    }
    return r;
}

}  // namespace k1
}  // namespace chip
