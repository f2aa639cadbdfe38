// secp256k1_host.hpp — constant-time secp256k1 scalar multiplication for the
// host ECIES stage (ecies 0.2 over libsecp256k1: encoding.rs:31-36,
// decoding.rs:62-69).
//
// OpenSSL has no dedicated secp256k1 code: its generic prime-field ladder set
// most of the latency of a small level-15 encode() (~450 us on the GPU box,
// DESIGN.md §6; ECIES does two scalar multiplications per encrypt and one
// per decrypt).  This is a small dedicated implementation (on the 2 GHz build
// container: k * P 194 us, k * G 53 us; ECIES encrypt 504 -> 401 us, decrypt
// 355 -> 261 us through the Python mirror):
//
//  * field elements: 4 x 64-bit limbs, products through unsigned __int128 and
//    carry chains through _addcarry_u64, reduced with 2^256 = 2^32 + 977
//    (mod p), always to [0, p); every function runs the same
//    instructions whatever the values (no branches or table indices on them);
//  * points: projective (X : Y : Z) with the complete formulas of Renes,
//    Costello and Batina (EUROCRYPT 2016), Algorithms 7 (addition) and 9
//    (doubling) for a = 0, b3 = 21.  They have no exceptional cases, so the
//    point at infinity and equal operands need no branches;
//  * k * P: fixed 4-bit windows (256 doublings, 64 additions); the window's
//    multiple is read by scanning the whole 16-entry table with masks;
//  * k * G: a precomputed table of i * 16^j * G (64 x 16 points, built once
//    per process), 64 additions and no doublings.
//
// Scalars are 32-byte big-endian with 0 < k < n (the caller checks, as
// libsecp256k1's SecretKey::parse).  tests/test_host_stages.py compares k * G
// and the ECIES envelopes (k * P inside) with the C and Python oracles'
// independent secp256k1 code on edge-case and random scalars.
#pragma once

#include <immintrin.h>

#include <cstdint>
#include <cstring>

namespace chip {
namespace k1 {

typedef unsigned __int128 u128;

struct Fe {
    uint64_t v[4];  // little-endian limbs, fully reduced (< p)
};

constexpr uint64_t RC = 0x1000003D1ull;  // 2^256 mod p
constexpr uint64_t P0 = 0xFFFFFFFEFFFFFC2Full, P1 = ~0ull, P2 = ~0ull, P3 = ~0ull;

// r[0..3] + hi * 2^256 (hi < 2^64) -> fully reduced.  Carry chains use the
// x86-64 add/sub-with-carry intrinsics (plain __int128 shifts compiled to a
// slow serial chain: 41 ns per addition).
inline void fe_reduce5(const uint64_t r[4], uint64_t hi, Fe &out) {
    unsigned long long a0, a1, a2, a3;
    const u128 m = (u128)hi * RC;
    unsigned char c = _addcarry_u64(0, r[0], (uint64_t)m, &a0);
    c = _addcarry_u64(c, r[1], (uint64_t)(m >> 64), &a1);
    c = _addcarry_u64(c, r[2], 0, &a2);
    c = _addcarry_u64(c, r[3], 0, &a3);
    // one more 2^256 (then a is small and this cannot carry out)
    unsigned char c2 = _addcarry_u64(0, a0, (uint64_t)c * RC, &a0);
    c2 = _addcarry_u64(c2, a1, 0, &a1);
    c2 = _addcarry_u64(c2, a2, 0, &a2);
    (void)_addcarry_u64(c2, a3, 0, &a3);
    // a < 2^256 < 2p: subtract p once if a >= p
    unsigned long long s0, s1, s2, s3;
    unsigned char b = _subborrow_u64(0, a0, P0, &s0);
    b = _subborrow_u64(b, a1, P1, &s1);
    b = _subborrow_u64(b, a2, P2, &s2);
    b = _subborrow_u64(b, a3, P3, &s3);
    const uint64_t keep = 0 - (uint64_t)b;  // all ones: a < p, keep a
    out.v[0] = (a0 & keep) | (s0 & ~keep);
    out.v[1] = (a1 & keep) | (s1 & ~keep);
    out.v[2] = (a2 & keep) | (s2 & ~keep);
    out.v[3] = (a3 & keep) | (s3 & ~keep);
}

inline Fe fe_mul(const Fe &a, const Fe &b) {
    uint64_t t[8];
    {  // schoolbook 4 x 4, row by row
        uint64_t carry = 0;
        for (int j = 0; j < 4; ++j) {
            const u128 acc = (u128)a.v[0] * b.v[j] + carry;
            t[j] = (uint64_t)acc;
            carry = (uint64_t)(acc >> 64);
        }
        t[4] = carry;
        for (int i = 1; i < 4; ++i) {
            carry = 0;
            for (int j = 0; j < 4; ++j) {
                const u128 acc = (u128)a.v[i] * b.v[j] + t[i + j] + carry;
                t[i + j] = (uint64_t)acc;
                carry = (uint64_t)(acc >> 64);
            }
            t[i + 4] = carry;
        }
    }
    // fold the high half: t_hi * 2^256 = t_hi * RC (RC < 2^33: each product < 2^97)
    uint64_t r[4];
    unsigned long long x;
    u128 p0 = (u128)t[4] * RC, p1 = (u128)t[5] * RC, p2 = (u128)t[6] * RC, p3 = (u128)t[7] * RC;
    unsigned char c = _addcarry_u64(0, t[0], (uint64_t)p0, &x);
    r[0] = x;
    c = _addcarry_u64(c, t[1], (uint64_t)p1, &x);
    unsigned char d = _addcarry_u64(0, x, (uint64_t)(p0 >> 64), &x);
    r[1] = x;
    c = _addcarry_u64(c, t[2], (uint64_t)p2, &x);
    d = _addcarry_u64(d, x, (uint64_t)(p1 >> 64), &x);
    r[2] = x;
    c = _addcarry_u64(c, t[3], (uint64_t)p3, &x);
    d = _addcarry_u64(d, x, (uint64_t)(p2 >> 64), &x);
    r[3] = x;
    const uint64_t hi = (uint64_t)(p3 >> 64) + c + d;
    Fe out;
    fe_reduce5(r, hi, out);
    return out;
}

inline Fe fe_sqr(const Fe &a) { return fe_mul(a, a); }

inline Fe fe_add(const Fe &a, const Fe &b) {
    unsigned long long r[4];
    unsigned char c = _addcarry_u64(0, a.v[0], b.v[0], &r[0]);
    c = _addcarry_u64(c, a.v[1], b.v[1], &r[1]);
    c = _addcarry_u64(c, a.v[2], b.v[2], &r[2]);
    c = _addcarry_u64(c, a.v[3], b.v[3], &r[3]);
    const uint64_t rr[4] = {r[0], r[1], r[2], r[3]};
    Fe out;
    fe_reduce5(rr, c, out);
    return out;
}

inline Fe fe_sub(const Fe &a, const Fe &b) {
    unsigned long long r[4];
    unsigned char bw = _subborrow_u64(0, a.v[0], b.v[0], &r[0]);
    bw = _subborrow_u64(bw, a.v[1], b.v[1], &r[1]);
    bw = _subborrow_u64(bw, a.v[2], b.v[2], &r[2]);
    bw = _subborrow_u64(bw, a.v[3], b.v[3], &r[3]);
    // a - b < 0: add p (the carry out of that addition is the wrap back)
    const uint64_t m = 0 - (uint64_t)bw;
    Fe out;
    unsigned long long x;
    unsigned char c = _addcarry_u64(0, r[0], P0 & m, &x);
    out.v[0] = x;
    c = _addcarry_u64(c, r[1], P1 & m, &x);
    out.v[1] = x;
    c = _addcarry_u64(c, r[2], P2 & m, &x);
    out.v[2] = x;
    (void)_addcarry_u64(c, r[3], P3 & m, &x);
    out.v[3] = x;
    return out;
}

inline Fe fe_mul21(const Fe &a) {  // b3 = 3 * 7
    uint64_t r[4];
    u128 acc = 0;
    for (int i = 0; i < 4; ++i) {
        acc = (acc >> 64) + (u128)a.v[i] * 21u;
        r[i] = (uint64_t)acc;
    }
    Fe out;
    fe_reduce5(r, (uint64_t)(acc >> 64), out);
    return out;
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

inline Fe fe_from_be(const uint8_t b[32]) {
    Fe f;
    for (int i = 0; i < 4; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
        f.v[i] = w;
    }
    return f;
}

inline void fe_to_be(const Fe &f, uint8_t b[32]) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(f.v[i] >> (56 - 8 * j));
}

struct Pt {
    Fe x, y, z;  // projective; infinity = (0 : 1 : 0)
};

inline Pt pt_inf() { return Pt{{{0, 0, 0, 0}}, {{1, 0, 0, 0}}, {{0, 0, 0, 0}}}; }

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
        for (int k = 0; k < 12; ++k) d[k] |= s[k] & m;
    }
    return r;
}

inline uint32_t nibble(const uint8_t k[32], int j) {  // j-th 4-bit window from the least significant end
    const uint8_t b = k[31 - j / 2];
    return (j & 1) ? (b >> 4) : (b & 15u);
}

// k * P for an affine point P = (x, y)
inline Pt mul(const uint8_t k[32], const Fe &x, const Fe &y) {
    Pt table[16];
    table[0] = pt_inf();
    table[1] = Pt{x, y, {{1, 0, 0, 0}}};
    for (int i = 2; i < 16; ++i) table[i] = pt_add(table[i - 1], table[1]);
    Pt r = pt_inf();
    for (int j = 63; j >= 0; --j) {
        r = pt_dbl(pt_dbl(pt_dbl(pt_dbl(r))));
        r = pt_add(r, pt_select(table, nibble(k, j)));
    }
    return r;
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

// i * 16^j * G for j < 64, i < 16 (built on first use, ~0.3 ms)
struct GTable {
    Pt t[64][16];
    GTable() {
        Pt base{gx(), gy(), {{1, 0, 0, 0}}};
        for (int j = 0; j < 64; ++j) {
            t[j][0] = pt_inf();
            t[j][1] = base;
            for (int i = 2; i < 16; ++i) t[j][i] = pt_add(t[j][i - 1], base);
            base = pt_dbl(pt_dbl(pt_dbl(pt_dbl(base))));
        }
    }
};

inline const GTable &gtable() {
    static const GTable *g = new GTable();  // never destroyed (used from host-stage threads)
    return *g;
}

inline Pt mul_g(const uint8_t k[32]) {
    const GTable &g = gtable();
    Pt r = pt_inf();
    for (int j = 0; j < 64; ++j) r = pt_add(r, pt_select(g.t[j], nibble(k, j)));
    return r;
}

// affine (x, y) of a point other than infinity, as 0x04 || x || y
inline bool to65(const Pt &p, uint8_t out[65]) {
    const Fe &z = p.z;
    if ((z.v[0] | z.v[1] | z.v[2] | z.v[3]) == 0) return false;  // infinity (public: a failed operation)
    const Fe zi = fe_inv(z);
    out[0] = 0x04;
    fe_to_be(fe_mul(p.x, zi), out + 1);
    fe_to_be(fe_mul(p.y, zi), out + 33);
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

}  // namespace k1
}  // namespace chip
