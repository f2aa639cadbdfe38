// gcm_vaes.cpp — see gcm_vaes.hpp.  GHASH works on byte-reversed blocks with
// the carry-less multiply, shift and two-phase reduction of Gueron and
// Kounavis ("Intel Carry-Less Multiplication Instruction and its Usage for
// Computing the GCM Mode", alg. 5); sixteen blocks share one reduction
// (their products with H^16 .. H^1 summed first, GHASH being linear).
#include "gcm_vaes.hpp"

#include <immintrin.h>

#include <cstring>

#define GCM_TARGET \
    __attribute__((target("aes,pclmul,sse4.1,ssse3,avx2,avx512f,avx512bw,avx512vl,avx512dq,vaes,vpclmulqdq")))

namespace chip {
namespace host {
namespace {

GCM_TARGET inline __m128i bswap128(__m128i x) {
    return _mm_shuffle_epi8(x, _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
}

GCM_TARGET inline __m128i ld(const uint8_t *p) { return _mm_loadu_si128(reinterpret_cast<const __m128i *>(p)); }
GCM_TARGET inline void st(uint8_t *p, __m128i x) { _mm_storeu_si128(reinterpret_cast<__m128i *>(p), x); }

// AES-256 key schedule with AESKEYGENASSIST (FIPS-197 §5.2)
GCM_TARGET inline __m128i exp_a(__m128i a, __m128i t) {
    t = _mm_shuffle_epi32(t, 0xff);
    a = _mm_xor_si128(a, _mm_slli_si128(a, 4));
    a = _mm_xor_si128(a, _mm_slli_si128(a, 4));
    a = _mm_xor_si128(a, _mm_slli_si128(a, 4));
    return _mm_xor_si128(a, t);
}
GCM_TARGET inline __m128i exp_b(__m128i b, __m128i t) {
    t = _mm_shuffle_epi32(t, 0xaa);
    b = _mm_xor_si128(b, _mm_slli_si128(b, 4));
    b = _mm_xor_si128(b, _mm_slli_si128(b, 4));
    b = _mm_xor_si128(b, _mm_slli_si128(b, 4));
    return _mm_xor_si128(b, t);
}

GCM_TARGET void expand256(const uint8_t *key, uint8_t (*rk)[16]) {
    __m128i a = ld(key), b = ld(key + 16);
    st(rk[0], a);
    st(rk[1], b);
#define CHIP_AES_STEP(i, rcon)                                \
    a = exp_a(a, _mm_aeskeygenassist_si128(b, rcon));         \
    st(rk[2 * (i)], a);                                       \
    if ((i) < 7) {                                            \
        b = exp_b(b, _mm_aeskeygenassist_si128(a, 0));        \
        st(rk[2 * (i) + 1], b);                               \
    }
    CHIP_AES_STEP(1, 0x01)
    CHIP_AES_STEP(2, 0x02)
    CHIP_AES_STEP(3, 0x04)
    CHIP_AES_STEP(4, 0x08)
    CHIP_AES_STEP(5, 0x10)
    CHIP_AES_STEP(6, 0x20)
    CHIP_AES_STEP(7, 0x40)
#undef CHIP_AES_STEP
}

GCM_TARGET inline __m128i aes_block(__m128i x, const uint8_t (*rk)[16]) {
    x = _mm_xor_si128(x, ld(rk[0]));
    for (int r = 1; r < 14; ++r) x = _mm_aesenc_si128(x, ld(rk[r]));
    return _mm_aesenclast_si128(x, ld(rk[14]));
}

// (hi:lo) + mid x^64, shifted left one bit (the operands are bit-reflected)
// and reduced modulo x^128 + x^7 + x^2 + x + 1
GCM_TARGET inline __m128i reduce(__m128i lo, __m128i mid, __m128i hi) {
    lo = _mm_xor_si128(lo, _mm_slli_si128(mid, 8));
    hi = _mm_xor_si128(hi, _mm_srli_si128(mid, 8));
    __m128i t7 = _mm_srli_epi32(lo, 31), t8 = _mm_srli_epi32(hi, 31);
    lo = _mm_slli_epi32(lo, 1);
    hi = _mm_slli_epi32(hi, 1);
    const __m128i t9 = _mm_srli_si128(t7, 12);
    t8 = _mm_slli_si128(t8, 4);
    t7 = _mm_slli_si128(t7, 4);
    lo = _mm_or_si128(lo, t7);
    hi = _mm_or_si128(hi, t8);
    hi = _mm_or_si128(hi, t9);
    t7 = _mm_xor_si128(_mm_xor_si128(_mm_slli_epi32(lo, 31), _mm_slli_epi32(lo, 30)), _mm_slli_epi32(lo, 25));
    t8 = _mm_srli_si128(t7, 4);
    t7 = _mm_slli_si128(t7, 12);
    lo = _mm_xor_si128(lo, t7);
    __m128i t2 = _mm_xor_si128(_mm_xor_si128(_mm_srli_epi32(lo, 1), _mm_srli_epi32(lo, 2)), _mm_srli_epi32(lo, 7));
    t2 = _mm_xor_si128(t2, t8);
    lo = _mm_xor_si128(lo, t2);
    return _mm_xor_si128(hi, lo);
}

GCM_TARGET inline __m128i gfmul(__m128i a, __m128i b) {
    const __m128i lo = _mm_clmulepi64_si128(a, b, 0x00), hi = _mm_clmulepi64_si128(a, b, 0x11);
    const __m128i mid = _mm_xor_si128(_mm_clmulepi64_si128(a, b, 0x10), _mm_clmulepi64_si128(a, b, 0x01));
    return reduce(lo, mid, hi);
}

GCM_TARGET inline __m128i xor4(__m512i v) {
    return _mm_xor_si128(_mm_xor_si128(_mm512_extracti32x4_epi32(v, 0), _mm512_extracti32x4_epi32(v, 1)),
                         _mm_xor_si128(_mm512_extracti32x4_epi32(v, 2), _mm512_extracti32x4_epi32(v, 3)));
}

inline void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24), p[1] = (uint8_t)(v >> 16), p[2] = (uint8_t)(v >> 8), p[3] = (uint8_t)v;
}

// nchunks x 256 bytes: 16 counter blocks through the four AES lanes, then
// their GHASH (over the ciphertext: `out` when encrypting, `in` when not)
GCM_TARGET void bulk(Gcm &g, const uint8_t *in, uint8_t *out, size_t nchunks) {
    __m512i rk[15];
    for (int r = 0; r < 15; ++r) rk[r] = _mm512_broadcast_i32x4(ld(g.rk[r]));
    const __m512i h0 = _mm512_loadu_si512(g.hp[0]), h1 = _mm512_loadu_si512(g.hp[4]);
    const __m512i h2 = _mm512_loadu_si512(g.hp[8]), h3 = _mm512_loadu_si512(g.hp[12]);
    const __m512i bsw = _mm512_broadcast_i32x4(_mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
    // counter blocks kept with the counter as a native dword 3 (the prefix in
    // dwords 0-2 as its bytes are), turned big-endian by one byte shuffle
    uint32_t pw[3];
    std::memcpy(pw, g.prefix, 12);
    const uint32_t c0 = g.ctr;
    __m512i cv[4];
    for (int q = 0; q < 4; ++q)
        cv[q] = _mm512_set_epi32((int)(c0 + 4 * q + 3), (int)pw[2], (int)pw[1], (int)pw[0], (int)(c0 + 4 * q + 2),
                                 (int)pw[2], (int)pw[1], (int)pw[0], (int)(c0 + 4 * q + 1), (int)pw[2], (int)pw[1],
                                 (int)pw[0], (int)(c0 + 4 * q), (int)pw[2], (int)pw[1], (int)pw[0]);
    const __m512i inc = _mm512_set_epi32(16, 0, 0, 0, 16, 0, 0, 0, 16, 0, 0, 0, 16, 0, 0, 0);
    const __m512i be = _mm512_broadcast_i32x4(_mm_set_epi8(12, 13, 14, 15, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0));
    __m128i y = ld(g.y);
    for (size_t c = 0; c < nchunks; ++c, in += 256, out += 256) {
        __m512i x0 = _mm512_xor_si512(_mm512_shuffle_epi8(cv[0], be), rk[0]);
        __m512i x1 = _mm512_xor_si512(_mm512_shuffle_epi8(cv[1], be), rk[0]);
        __m512i x2 = _mm512_xor_si512(_mm512_shuffle_epi8(cv[2], be), rk[0]);
        __m512i x3 = _mm512_xor_si512(_mm512_shuffle_epi8(cv[3], be), rk[0]);
        for (int q = 0; q < 4; ++q) cv[q] = _mm512_add_epi32(cv[q], inc);
        for (int r = 1; r < 14; ++r) {
            x0 = _mm512_aesenc_epi128(x0, rk[r]);
            x1 = _mm512_aesenc_epi128(x1, rk[r]);
            x2 = _mm512_aesenc_epi128(x2, rk[r]);
            x3 = _mm512_aesenc_epi128(x3, rk[r]);
        }
        x0 = _mm512_aesenclast_epi128(x0, rk[14]);
        x1 = _mm512_aesenclast_epi128(x1, rk[14]);
        x2 = _mm512_aesenclast_epi128(x2, rk[14]);
        x3 = _mm512_aesenclast_epi128(x3, rk[14]);
        const __m512i d0 = _mm512_loadu_si512(in), d1 = _mm512_loadu_si512(in + 64);
        const __m512i d2 = _mm512_loadu_si512(in + 128), d3 = _mm512_loadu_si512(in + 192);
        const __m512i o0 = _mm512_xor_si512(d0, x0), o1 = _mm512_xor_si512(d1, x1);
        const __m512i o2 = _mm512_xor_si512(d2, x2), o3 = _mm512_xor_si512(d3, x3);
        _mm512_storeu_si512(out, o0);
        _mm512_storeu_si512(out + 64, o1);
        _mm512_storeu_si512(out + 128, o2);
        _mm512_storeu_si512(out + 192, o3);
        __m512i g0 = _mm512_shuffle_epi8(g.enc ? o0 : d0, bsw), g1 = _mm512_shuffle_epi8(g.enc ? o1 : d1, bsw);
        __m512i g2 = _mm512_shuffle_epi8(g.enc ? o2 : d2, bsw), g3 = _mm512_shuffle_epi8(g.enc ? o3 : d3, bsw);
        g0 = _mm512_xor_si512(g0, _mm512_zextsi128_si512(y));
        __m512i lo = _mm512_xor_si512(
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g0, h0, 0x00), _mm512_clmulepi64_epi128(g1, h1, 0x00)),
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g2, h2, 0x00), _mm512_clmulepi64_epi128(g3, h3, 0x00)));
        __m512i hi = _mm512_xor_si512(
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g0, h0, 0x11), _mm512_clmulepi64_epi128(g1, h1, 0x11)),
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g2, h2, 0x11), _mm512_clmulepi64_epi128(g3, h3, 0x11)));
        __m512i mid = _mm512_xor_si512(
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g0, h0, 0x01), _mm512_clmulepi64_epi128(g0, h0, 0x10)),
            _mm512_xor_si512(_mm512_clmulepi64_epi128(g1, h1, 0x01), _mm512_clmulepi64_epi128(g1, h1, 0x10)));
        mid = _mm512_xor_si512(
            mid, _mm512_xor_si512(
                     _mm512_xor_si512(_mm512_clmulepi64_epi128(g2, h2, 0x01), _mm512_clmulepi64_epi128(g2, h2, 0x10)),
                     _mm512_xor_si512(_mm512_clmulepi64_epi128(g3, h3, 0x01), _mm512_clmulepi64_epi128(g3, h3, 0x10))));
        y = reduce(xor4(lo), xor4(mid), xor4(hi));
    }
    st(g.y, y);
    g.ctr = c0 + (uint32_t)(16 * nchunks);
}

// one counter block's keystream (bytes 12..15: big-endian counter)
GCM_TARGET __m128i keystream(Gcm &g) {
    alignas(16) uint8_t b[16];
    std::memcpy(b, g.prefix, 12);
    put_be32(b + 12, g.ctr++);
    return aes_block(_mm_load_si128(reinterpret_cast<const __m128i *>(b)), g.rk);
}

GCM_TARGET void ghash_block(Gcm &g, const uint8_t *blk) {
    st(g.y, gfmul(_mm_xor_si128(ld(g.y), bswap128(ld(blk))), ld(g.hp[15])));
}

GCM_TARGET void init_impl(Gcm &g, const uint8_t *key, const uint8_t *iv, size_t ivlen, bool encrypt) {
    expand256(key, g.rk);
    const __m128i h = bswap128(aes_block(_mm_setzero_si128(), g.rk));
    __m128i p = h;
    st(g.hp[15], p);
    for (int k = 2; k <= 16; ++k) {
        p = gfmul(p, h);
        st(g.hp[16 - k], p);
    }
    st(g.y, _mm_setzero_si128());
    if (ivlen == 12) {
        std::memcpy(g.j0, iv, 12);
        put_be32(g.j0 + 12, 1);
    } else {  // J0 = GHASH(IV || 0-pad || [0]_64 || [len(IV)]_64)
        uint8_t blk[16];
        size_t o = 0;
        for (; o + 16 <= ivlen; o += 16) ghash_block(g, iv + o);
        if (o < ivlen) {
            std::memset(blk, 0, 16);
            std::memcpy(blk, iv + o, ivlen - o);
            ghash_block(g, blk);
        }
        std::memset(blk, 0, 8);
        const uint64_t bits = (uint64_t)ivlen * 8;
        for (int i = 0; i < 8; ++i) blk[8 + i] = (uint8_t)(bits >> (56 - 8 * i));
        ghash_block(g, blk);
        st(g.j0, bswap128(ld(g.y)));
        st(g.y, _mm_setzero_si128());
    }
    std::memcpy(g.prefix, g.j0, 12);
    g.ctr = ((uint32_t)g.j0[12] << 24 | (uint32_t)g.j0[13] << 16 | (uint32_t)g.j0[14] << 8 | g.j0[15]) + 1;
    g.npend = 0;
    g.len = 0;
    g.enc = encrypt;
}

GCM_TARGET void update_impl(Gcm &g, const uint8_t *in, size_t n, uint8_t *out) {
    g.len += n;
    while (g.npend && n) {  // the partial block's keystream first
        const uint8_t c = in[0] ^ g.ks[g.npend];
        out[0] = c;
        g.pend[g.npend++] = g.enc ? c : in[0];
        ++in, ++out, --n;
        if (g.npend == 16) {
            ghash_block(g, g.pend);
            g.npend = 0;
        }
    }
    const size_t chunks = n / 256;
    if (chunks) {
        bulk(g, in, out, chunks);
        in += 256 * chunks, out += 256 * chunks, n -= 256 * chunks;
    }
    while (n >= 16) {
        const __m128i x = ld(in), o = _mm_xor_si128(x, keystream(g));
        st(out, o);
        st(g.y, gfmul(_mm_xor_si128(ld(g.y), bswap128(g.enc ? o : x)), ld(g.hp[15])));
        in += 16, out += 16, n -= 16;
    }
    if (n) {
        st(g.ks, keystream(g));
        for (size_t i = 0; i < n; ++i) {
            const uint8_t c = in[i] ^ g.ks[i];
            out[i] = c;
            g.pend[i] = g.enc ? c : in[i];
        }
        g.npend = (uint32_t)n;
    }
}

GCM_TARGET void tag_impl(Gcm &g, uint8_t out[16]) {
    if (g.npend) {
        std::memset(g.pend + g.npend, 0, 16 - g.npend);
        ghash_block(g, g.pend);
        g.npend = 0;
    }
    uint8_t blk[16] = {0};
    const uint64_t bits = g.len * 8;
    for (int i = 0; i < 8; ++i) blk[8 + i] = (uint8_t)(bits >> (56 - 8 * i));
    ghash_block(g, blk);
    const __m128i s = bswap128(ld(g.y));
    st(out, _mm_xor_si128(s, aes_block(ld(g.j0), g.rk)));
}

// H^k (k >= 1) in the byte-reversed representation, by square and multiply
GCM_TARGET __m128i h_pow(const Gcm &g, uint64_t k) {
    __m128i r = ld(g.hp[15]), b = r;  // H
    bool have = false;
    for (; k; k >>= 1) {
        if (k & 1) {
            r = have ? gfmul(r, b) : b;
            have = true;
        }
        if (k > 1) b = gfmul(b, b);
    }
    return r;
}

GCM_TARGET void join_impl(Gcm &g, const uint8_t *yp, uint64_t blocks_after) {
    __m128i y = ld(yp);
    if (blocks_after) y = gfmul(y, h_pow(g, blocks_after));
    st(g.y, _mm_xor_si128(ld(g.y), y));
}

}  // namespace

void Gcm::init_part(const Gcm &msg, uint64_t offset) {
    std::memcpy(rk, msg.rk, sizeof rk);
    std::memcpy(hp, msg.hp, sizeof hp);
    std::memcpy(j0, msg.j0, sizeof j0);
    std::memcpy(prefix, msg.prefix, sizeof prefix);
    const uint32_t c0 = ((uint32_t)j0[12] << 24 | (uint32_t)j0[13] << 16 | (uint32_t)j0[14] << 8 | j0[15]) + 1;
    ctr = c0 + (uint32_t)(offset / 16);  // inc32: the counter wraps in its 32 bits
    std::memset(y, 0, sizeof y);
    npend = 0;
    len = 0;
    enc = msg.enc;
}
void Gcm::part_ghash(uint8_t out[16]) {
    if (npend) {
        std::memset(pend + npend, 0, 16 - npend);
        ghash_block(*this, pend);
        npend = 0;
    }
    std::memcpy(out, y, 16);
}
void Gcm::join_part(const uint8_t y_part[16], uint64_t blocks_after) { join_impl(*this, y_part, blocks_after); }
void Gcm::tag_joined(uint64_t total, uint8_t out[16]) {
    npend = 0;
    len = total;
    tag_impl(*this, out);
}

void Gcm::init(const uint8_t *key, const uint8_t *iv, size_t ivlen, bool encrypt) {
    init_impl(*this, key, iv, ivlen, encrypt);
}
bool Gcm::update(const uint8_t *in, size_t n, uint8_t *out) {
    if (n > GCM_MAX_BYTES - len) return false;
    update_impl(*this, in, n, out);
    return true;
}
void Gcm::tag(uint8_t out[16]) { tag_impl(*this, out); }
void Gcm::wipe() {
    volatile uint8_t *p = reinterpret_cast<volatile uint8_t *>(this);
    for (size_t i = 0; i < sizeof(*this); ++i) p[i] = 0;
}

bool gcm_fast_available() {
    static const bool ok = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("aes") && __builtin_cpu_supports("pclmul") &&
               __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
               __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq") &&
               __builtin_cpu_supports("vaes") && __builtin_cpu_supports("vpclmulqdq");
    }();
    return ok;
}

}  // namespace host
}  // namespace chip
