/*
 * host_oracle.c — TEST INFRASTRUCTURE ONLY: plain-C restatement of the host
 * stages of carbonado encode()/decode() (snappy framing, ECIES), used by the
 * tests as a fast full-size checker and by bench.py as the CPU baseline of the
 * level-15 pipeline.  Never linked into the product.
 *
 * References (reference crate call sites; the crates themselves are absent):
 *   encoding::snap  /root/reference/src/encoding.rs:16-28  (snap 1.1 FrameEncoder)
 *   encoding::ecies /root/reference/src/encoding.rs:30-36  (ecies 0.2.6 encrypt)
 *   decoding::ecies /root/reference/src/decoding.rs:62-68
 *   decoding::snap  /root/reference/src/decoding.rs:70-77
 * Restated algorithms: snappy framing format + Go snappy encodeBlock;
 * FIPS 180-4 SHA-256; RFC 2104 HMAC; RFC 5869 HKDF; FIPS-197 AES-256;
 * SP 800-38D GCM (4-bit-table GHASH); SEC 2 secp256k1 (Jacobian
 * coordinates, 4x64-bit limbs).  Pinned by tests/golden/host_kat.json and by
 * oracle/host_oracle.py (independent Python restatement).
 */
#include "carbonado_oracle.h"

#include <stdlib.h>
#include <string.h>

__extension__ typedef unsigned __int128 u128;

/* ------------------------------------------------------------ CRC-32C */
static uint32_t crc_tab[256];
static int crc_ready;

static void crc_init(void) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_tab[i] = c;
    }
    crc_ready = 1;
}

uint32_t orc_crc32c(const uint8_t *p, uint64_t n) {
    if (!crc_ready) crc_init();
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; ++i) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

static uint32_t crc_masked(const uint8_t *p, uint64_t n) {
    uint32_t c = orc_crc32c(p, n);
    return ((c >> 15) | (c << 17)) + 0xA282EAD8u;
}

/* ------------------------------------------------------------ snappy */
#define SNAP_BLOCK 65536u
static const uint8_t SNAP_ID[10] = {0xFF, 0x06, 0x00, 0x00, 's', 'N', 'a', 'P', 'p', 'Y'};

static uint32_t ld32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

static uint64_t lit(uint8_t *d, const uint8_t *s, uint64_t len) {
    uint64_t n = len - 1, i;
    if (n < 60) { d[0] = (uint8_t)(n << 2); i = 1; }
    else if (n < 256) { d[0] = 60 << 2; d[1] = (uint8_t)n; i = 2; }
    else { d[0] = 61 << 2; d[1] = (uint8_t)n; d[2] = (uint8_t)(n >> 8); i = 3; }
    memcpy(d + i, s, len);
    return i + len;
}

static uint64_t cpy(uint8_t *d, uint64_t off, uint64_t len) {
    uint64_t i = 0;
    for (; len >= 68; len -= 64, i += 3) { d[i] = (63 << 2) | 2; d[i + 1] = (uint8_t)off; d[i + 2] = (uint8_t)(off >> 8); }
    if (len > 64) { d[i] = (59 << 2) | 2; d[i + 1] = (uint8_t)off; d[i + 2] = (uint8_t)(off >> 8); i += 3; len -= 60; }
    if (len >= 12 || off >= 2048) {
        d[i] = (uint8_t)(((len - 1) << 2) | 2); d[i + 1] = (uint8_t)off; d[i + 2] = (uint8_t)(off >> 8);
        return i + 3;
    }
    d[i] = (uint8_t)(((off >> 8) << 5) | ((len - 4) << 2) | 1); d[i + 1] = (uint8_t)off;
    return i + 2;
}

/* raw snappy of one block (<= 64 KiB) including the varint length */
static uint64_t snap_block(uint8_t *d, const uint8_t *s, uint64_t n) {
    uint64_t o = 0, v = n;
    if (n == 0) { d[0] = 0; return 1; }
    while (v >= 0x80) { d[o++] = (uint8_t)(v | 0x80); v >>= 7; }
    d[o++] = (uint8_t)v;
    if (n < 17) return o + lit(d + o, s, n);
    unsigned shift = 24;
    uint64_t ts = 256;
    while (ts < 16384 && ts < n) { --shift; ts <<= 1; }
    uint16_t table[16384]; /* per call: the oracle runs on many threads at once */
    memset(table, 0, ts * sizeof(uint16_t));
#define HSH(u) ((uint32_t)((uint32_t)(u) * 0x1E35A7BDu) >> shift)
    const uint64_t lim = n - 15;
    uint64_t emit = 0, p = 1, cand = 0;
    uint32_t nh = HSH(ld32(s + 1));
    for (;;) {
        uint64_t skip = 32, pn = p;
        for (;;) {
            p = pn;
            uint64_t step = skip >> 5;
            pn = p + step;
            skip += step;
            if (pn > lim) goto rest;
            cand = table[nh];
            table[nh] = (uint16_t)p;
            nh = HSH(ld32(s + pn));
            if (ld32(s + p) == ld32(s + cand)) break;
        }
        o += lit(d + o, s + emit, p - emit);
        for (;;) {
            uint64_t base = p;
            p += 4;
            for (uint64_t i = cand + 4; p < n && s[i] == s[p]; ++i, ++p) {}
            o += cpy(d + o, base - cand, p - base);
            emit = p;
            if (p >= lim) goto rest;
            table[HSH(ld32(s + p - 1))] = (uint16_t)(p - 1);
            uint32_t ch = HSH(ld32(s + p));
            cand = table[ch];
            table[ch] = (uint16_t)p;
            if (ld32(s + p) != ld32(s + cand)) { nh = HSH(ld32(s + p + 1)); ++p; break; }
        }
    }
rest:
    if (emit < n) o += lit(d + o, s + emit, n - emit);
#undef HSH
    return o;
}

uint64_t orc_snap_max_len(uint64_t n) { return n ? 10 + 8 * ((n + SNAP_BLOCK - 1) / SNAP_BLOCK) + n : 0; }

int orc_snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (n == 0) { *out_len = 0; return ORC_OK; }
    if (cap < orc_snap_max_len(n)) return ORC_ERR_BUFFER_TOO_SMALL;
    uint8_t *tmp = (uint8_t *)malloc(32 + SNAP_BLOCK + SNAP_BLOCK / 6);
    if (!tmp) return ORC_ERR_INVALID_ARG;
    uint64_t o = 10;
    memcpy(out, SNAP_ID, 10);
    for (uint64_t b = 0; b < n; b += SNAP_BLOCK) {
        uint64_t len = n - b < SNAP_BLOCK ? n - b : SNAP_BLOCK;
        uint32_t crc = crc_masked(in + b, len);
        uint64_t cl = snap_block(tmp, in + b, len);
        int raw = cl >= len - len / 8;
        uint64_t body = raw ? len : cl, clen = 4 + body;
        out[o] = raw ? 1 : 0; out[o + 1] = (uint8_t)clen; out[o + 2] = (uint8_t)(clen >> 8); out[o + 3] = (uint8_t)(clen >> 16);
        out[o + 4] = (uint8_t)crc; out[o + 5] = (uint8_t)(crc >> 8); out[o + 6] = (uint8_t)(crc >> 16); out[o + 7] = (uint8_t)(crc >> 24);
        memcpy(out + o + 8, raw ? in + b : tmp, body);
        o += 8 + body;
    }
    free(tmp);
    *out_len = o;
    return ORC_OK;
}

static int snap_unblock(const uint8_t *s, uint64_t n, uint8_t *d, uint64_t cap, uint64_t *dl) {
    uint64_t len = 0, i = 0, o = 0;
    for (unsigned sh = 0;; sh += 7) {
        if (i >= n || sh > 63) return ORC_ERR_SNAP;
        len |= (uint64_t)(s[i] & 0x7F) << sh;
        if (!(s[i++] & 0x80)) break;
    }
    if (len > cap) return ORC_ERR_SNAP;
    while (i < n) {
        uint8_t t = s[i];
        uint64_t l, off;
        if ((t & 3) == 0) {
            l = t >> 2;
            if (l < 60) ++i;
            else {
                unsigned nb = (unsigned)(l - 59);
                if (i + 1 + nb > n) return ORC_ERR_SNAP;
                l = 0;
                for (unsigned b = 0; b < nb; ++b) l |= (uint64_t)s[i + 1 + b] << (8 * b);
                i += 1 + nb;
            }
            ++l;
            if (l > n - i || l > len - o) return ORC_ERR_SNAP;
            memcpy(d + o, s + i, l);
            i += l; o += l;
            continue;
        }
        if ((t & 3) == 1) { if (i + 2 > n) return ORC_ERR_SNAP; l = 4 + ((t >> 2) & 7); off = ((uint64_t)(t >> 5) << 8) | s[i + 1]; i += 2; }
        else if ((t & 3) == 2) { if (i + 3 > n) return ORC_ERR_SNAP; l = 1 + (t >> 2); off = s[i + 1] | (uint64_t)s[i + 2] << 8; i += 3; }
        else { if (i + 5 > n) return ORC_ERR_SNAP; l = 1 + (t >> 2); off = ld32(s + i + 1); i += 5; }
        if (off == 0 || off > o || l > len - o) return ORC_ERR_SNAP;
        for (uint64_t k = 0; k < l; ++k, ++o) d[o] = d[o - off];
    }
    if (o != len) return ORC_ERR_SNAP;
    *dl = o;
    return ORC_OK;
}

int orc_snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    uint64_t i = 0, o = 0;
    int ident = 0;
    while (i < n) {
        if (n - i < 4) return ORC_ERR_SNAP;
        uint8_t ty = in[i];
        uint64_t cl = in[i + 1] | (uint64_t)in[i + 2] << 8 | (uint64_t)in[i + 3] << 16;
        i += 4;
        if (cl > n - i) return ORC_ERR_SNAP;
        const uint8_t *b = in + i;
        if (!ident && ty != 0xFF) return ORC_ERR_SNAP;
        if (ty == 0xFF) {
            if (cl != 6 || memcmp(b, SNAP_ID + 4, 6)) return ORC_ERR_SNAP;
            ident = 1;
        } else if (ty == 0 || ty == 1) {
            if (cl < 4) return ORC_ERR_SNAP;
            uint32_t want = ld32(b);
            uint64_t dl = cl - 4;
            if (ty == 1) {
                if (dl > SNAP_BLOCK || dl > cap - o) return ORC_ERR_SNAP;
                memcpy(out + o, b + 4, dl);
            } else {
                uint64_t room = cap - o < SNAP_BLOCK ? cap - o : SNAP_BLOCK;
                int rc = snap_unblock(b + 4, dl, out + o, room, &dl);
                if (rc) return rc;
            }
            if (crc_masked(out + o, dl) != want) return ORC_ERR_SNAP;
            o += dl;
        } else if (ty >= 0x02 && ty <= 0x7F) {
            return ORC_ERR_SNAP;
        }
        i += cl;
    }
    *out_len = o;
    return ORC_OK;
}

/* ------------------------------------------------------------ SHA-256 / HMAC / HKDF */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t rr(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

static void sha_block(uint32_t h[8], const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i)
        w[i] = w[i - 16] + (rr(w[i - 15], 7) ^ rr(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
               (rr(w[i - 2], 17) ^ rr(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = k + (rr(e, 6) ^ rr(e, 11) ^ rr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rr(a, 2) ^ rr(a, 13) ^ rr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

/* SHA-256 of the concatenation of two buffers */
static void sha256_2(const uint8_t *a, uint64_t na, const uint8_t *b, uint64_t nb, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[128];
    uint64_t fill = 0, total = na + nb;
    const uint8_t *src[2] = {a, b};
    uint64_t len[2] = {na, nb};
    for (int s = 0; s < 2; ++s)
        for (uint64_t i = 0; i < len[s]; ++i) {
            buf[fill++] = src[s][i];
            if (fill == 64) { sha_block(h, buf); fill = 0; }
        }
    buf[fill++] = 0x80;
    if (fill > 56) { memset(buf + fill, 0, 64 - fill); sha_block(h, buf); fill = 0; }
    memset(buf + fill, 0, 56 - fill);
    for (int i = 0; i < 8; ++i) buf[56 + i] = (uint8_t)((total * 8) >> (56 - 8 * i));
    sha_block(h, buf);
    for (int i = 0; i < 8; ++i) { out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16); out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i]; }
}

void orc_sha256(const uint8_t *in, uint64_t n, uint8_t out[32]) { sha256_2(in, n, NULL, 0, out); }

void orc_hmac_sha256(const uint8_t *key, uint64_t kl, const uint8_t *msg, uint64_t n, uint8_t out[32]) {
    uint8_t k[64] = {0}, ipad[64], opad[64], inner[32];
    if (kl > 64) orc_sha256(key, kl, k); else memcpy(k, key, kl);
    for (int i = 0; i < 64; ++i) { ipad[i] = k[i] ^ 0x36; opad[i] = k[i] ^ 0x5C; }
    sha256_2(ipad, 64, msg, n, inner);
    sha256_2(opad, 64, inner, 32, out);
}

/* HKDF-SHA256, no salt, no info, 32 bytes (ecies hkdf_sha256) */
static void hkdf32(const uint8_t *ikm, uint64_t n, uint8_t out[32]) {
    uint8_t zero[32] = {0}, prk[32], one = 1;
    orc_hmac_sha256(zero, 32, ikm, n, prk);
    orc_hmac_sha256(prk, 32, &one, 1, out);
}

/* ------------------------------------------------------------ AES-256 */
static uint8_t SB[256];
static uint32_t TE[4][256];
static int aes_ready;

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }

static void aes_init(void) {
    uint8_t p = 1, q = 1;
    do { /* p walks the multiplicative group by x3, q by its inverse */
        p = p ^ (uint8_t)(p << 1) ^ ((p & 0x80) ? 0x1B : 0);
        q ^= q << 1; q ^= q << 2; q ^= q << 4; if (q & 0x80) q ^= 0x09;
        uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        SB[p] = x ^ 0x63;
    } while (p != 1);
    SB[0] = 0x63;
    for (int i = 0; i < 256; ++i) {
        uint8_t s = SB[i], s2 = xt(s), s3 = s2 ^ s;
        uint32_t t = (uint32_t)s2 << 24 | (uint32_t)s << 16 | (uint32_t)s << 8 | s3;
        TE[0][i] = t; TE[1][i] = rr(t, 8); TE[2][i] = rr(t, 16); TE[3][i] = rr(t, 24);
    }
    aes_ready = 1;
}

/* the lazily built tables are built once at load time, before any thread
   runs (the checkers call the oracle from many threads) */
__attribute__((constructor)) static void host_oracle_tables(void) {
    crc_init();
    aes_init();
}

typedef struct { uint32_t rk[60]; } aes256;

static void aes_key(aes256 *a, const uint8_t key[32]) {
    if (!aes_ready) aes_init();
    uint32_t *w = a->rk;
    for (int i = 0; i < 8; ++i) w[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    uint8_t rc = 1;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = w[i - 1];
        if (i % 8 == 0) {
            t = rr(t, 24);
            t = (uint32_t)SB[t >> 24] << 24 | (uint32_t)SB[(t >> 16) & 0xFF] << 16 | (uint32_t)SB[(t >> 8) & 0xFF] << 8 | SB[t & 0xFF];
            t ^= (uint32_t)rc << 24;
            rc = xt(rc);
        } else if (i % 8 == 4) {
            t = (uint32_t)SB[t >> 24] << 24 | (uint32_t)SB[(t >> 16) & 0xFF] << 16 | (uint32_t)SB[(t >> 8) & 0xFF] << 8 | SB[t & 0xFF];
        }
        w[i] = w[i - 8] ^ t;
    }
}

static void aes_enc(const aes256 *a, const uint8_t in[16], uint8_t out[16]) {
    const uint32_t *k = a->rk;
    uint32_t s[4], t[4];
    for (int i = 0; i < 4; ++i) s[i] = ((uint32_t)in[4 * i] << 24 | (uint32_t)in[4 * i + 1] << 16 | (uint32_t)in[4 * i + 2] << 8 | in[4 * i + 3]) ^ k[i];
    for (int r = 1; r < 14; ++r) {
        for (int i = 0; i < 4; ++i)
            t[i] = TE[0][s[i] >> 24] ^ TE[1][(s[(i + 1) & 3] >> 16) & 0xFF] ^ TE[2][(s[(i + 2) & 3] >> 8) & 0xFF] ^
                   TE[3][s[(i + 3) & 3] & 0xFF] ^ k[4 * r + i];
        memcpy(s, t, sizeof s);
    }
    for (int i = 0; i < 4; ++i) {
        uint32_t v = ((uint32_t)SB[s[i] >> 24] << 24 | (uint32_t)SB[(s[(i + 1) & 3] >> 16) & 0xFF] << 16 |
                      (uint32_t)SB[(s[(i + 2) & 3] >> 8) & 0xFF] << 8 | SB[s[(i + 3) & 3] & 0xFF]) ^ k[56 + i];
        out[4 * i] = (uint8_t)(v >> 24); out[4 * i + 1] = (uint8_t)(v >> 16); out[4 * i + 2] = (uint8_t)(v >> 8); out[4 * i + 3] = (uint8_t)v;
    }
}

/* ------------------------------------------------------------ GCM */
typedef struct { uint64_t HL[16], HH[16]; } ghash_t;
static const uint64_t LAST4[16] = {0x0000, 0x1c20, 0x3840, 0x2460, 0x7080, 0x6ca0, 0x48c0, 0x54e0,
                                   0xe100, 0xfd20, 0xd940, 0xc560, 0x9180, 0x8da0, 0xa9c0, 0xb5e0};

static uint64_t be64(const uint8_t *p) { uint64_t v = 0; for (int i = 0; i < 8; ++i) v = v << 8 | p[i]; return v; }
static void put64(uint8_t *p, uint64_t v) { for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; } }

static void ghash_init(ghash_t *g, const uint8_t H[16]) {
    uint64_t vh = be64(H), vl = be64(H + 8);
    g->HL[0] = g->HH[0] = 0;
    g->HL[8] = vl; g->HH[8] = vh;
    for (int i = 4; i > 0; i >>= 1) {
        uint64_t T = (vl & 1) ? 0xe100000000000000ull : 0;
        vl = (vh << 63) | (vl >> 1);
        vh = (vh >> 1) ^ T;
        g->HL[i] = vl; g->HH[i] = vh;
    }
    for (int i = 2; i <= 8; i *= 2)
        for (int j = 1; j < i; ++j) { g->HH[i + j] = g->HH[i] ^ g->HH[j]; g->HL[i + j] = g->HL[i] ^ g->HL[j]; }
}

/* x <- x * H */
static void ghash_mul(const ghash_t *g, uint8_t x[16]) {
    uint8_t lo = x[15] & 0xF;
    uint64_t zh = g->HH[lo], zl = g->HL[lo];
    for (int i = 15; i >= 0; --i) {
        lo = x[i] & 0xF;
        uint8_t hi = x[i] >> 4, rem;
        if (i != 15) {
            rem = zl & 0xF;
            zl = (zh << 60) | (zl >> 4); zh = (zh >> 4) ^ (LAST4[rem] << 48);
            zh ^= g->HH[lo]; zl ^= g->HL[lo];
        }
        rem = zl & 0xF;
        zl = (zh << 60) | (zl >> 4); zh = (zh >> 4) ^ (LAST4[rem] << 48);
        zh ^= g->HH[hi]; zl ^= g->HL[hi];
    }
    put64(x, zh); put64(x + 8, zl);
}

static void ghash_update(const ghash_t *g, uint8_t y[16], const uint8_t *p, uint64_t n) {
    for (uint64_t o = 0; o < n; o += 16) {
        uint64_t l = n - o < 16 ? n - o : 16;
        for (uint64_t i = 0; i < l; ++i) y[i] ^= p[o + i];
        ghash_mul(g, y);
    }
}

static void inc32(uint8_t cb[16]) { for (int i = 15; i >= 12; --i) if (++cb[i]) break; }

/* AES-256-GCM with a 16-byte IV and no AAD; dec != 0 verifies `tag` first */
static int gcm(const uint8_t key[32], const uint8_t iv[16], const uint8_t *in, uint64_t n, uint8_t *out,
               uint8_t tag[16], int dec) {
    aes256 a;
    ghash_t g;
    uint8_t H[16] = {0}, j0[16] = {0}, lenblk[16] = {0}, s[16] = {0}, cb[16], ks[16], t[16];
    aes_key(&a, key);
    aes_enc(&a, H, H);
    ghash_init(&g, H);
    ghash_update(&g, j0, iv, 16); /* J0 = GHASH(IV || 0^64 || [128]_64) */
    put64(lenblk + 8, 128);
    ghash_update(&g, j0, lenblk, 16);
    if (dec) ghash_update(&g, s, in, n);
    memcpy(cb, j0, 16);
    for (uint64_t o = 0; o < n; o += 16) {
        inc32(cb);
        aes_enc(&a, cb, ks);
        uint64_t l = n - o < 16 ? n - o : 16;
        for (uint64_t i = 0; i < l; ++i) out[o + i] = in[o + i] ^ ks[i];
    }
    if (!dec) ghash_update(&g, s, out, n);
    memset(lenblk, 0, 16);
    put64(lenblk + 8, n * 8);
    ghash_update(&g, s, lenblk, 16);
    aes_enc(&a, j0, t);
    for (int i = 0; i < 16; ++i) t[i] ^= s[i];
    if (!dec) { memcpy(tag, t, 16); return ORC_OK; }
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i) diff |= (uint8_t)(t[i] ^ tag[i]);
    if (diff) { memset(out, 0, n); return ORC_ERR_ECIES; }
    return ORC_OK;
}

/* ------------------------------------------------------------ secp256k1 */
typedef struct { uint64_t v[4]; } fe; /* little-endian limbs, value < p */
static const fe FP = {{0xFFFFFFFEFFFFFC2Full, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull}};
static const uint8_t ORDER[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE,
                                  0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48, 0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};
static const uint8_t GXB[32] = {0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
                                0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
static const uint8_t GYB[32] = {0x48, 0x3A, 0xDA, 0x77, 0x26, 0xA3, 0xC4, 0x65, 0x5D, 0xA4, 0xFB, 0xFC, 0x0E, 0x11, 0x08, 0xA8,
                                0xFD, 0x17, 0xB4, 0x48, 0xA6, 0x85, 0x54, 0x19, 0x9C, 0x47, 0xD0, 0x8F, 0xFB, 0x10, 0xD4, 0xB8};

static int fe_geq_p(const fe *a) {
    for (int i = 3; i >= 0; --i) {
        if (a->v[i] > FP.v[i]) return 1;
        if (a->v[i] < FP.v[i]) return 0;
    }
    return 1;
}
static void fe_sub_p(fe *a) {
    u128 b = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->v[i] - FP.v[i] - b;
        a->v[i] = (uint64_t)d;
        b = (d >> 64) & 1;
    }
}
static void fe_add(fe *r, const fe *a, const fe *b) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    if (c || fe_geq_p(r)) fe_sub_p(r); /* 2^256 wrap: subtracting p mod 2^256 is the same as adding 2^32+977 */
}
static void fe_sub(fe *r, const fe *a, const fe *b) {
    u128 br = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->v[i] - b->v[i] - br;
        r->v[i] = (uint64_t)d;
        br = (d >> 64) & 1;
    }
    if (br) { /* add p */
        u128 c = 0;
        for (int i = 0; i < 4; ++i) { c += (u128)r->v[i] + FP.v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    }
}
static void fe_mul(fe *r, const fe *a, const fe *b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; j < 4; ++j) {
            c += (u128)a->v[i] * b->v[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    /* 2^256 = 0x1000003D1 (mod p): fold the high half twice */
    const uint64_t C = 0x1000003D1ull;
    u128 c = 0;
    uint64_t u[5];
    for (int i = 0; i < 4; ++i) { c += (u128)t[i + 4] * C + t[i]; u[i] = (uint64_t)c; c >>= 64; }
    u[4] = (uint64_t)c;
    c = (u128)u[4] * C;
    for (int i = 0; i < 4; ++i) { c += u[i]; r->v[i] = (uint64_t)c; c >>= 64; }
    if (c) { /* one more 2^256 */
        u128 d = (u128)r->v[0] + C;
        r->v[0] = (uint64_t)d;
        d >>= 64;
        for (int i = 1; i < 4 && d; ++i) { d += r->v[i]; r->v[i] = (uint64_t)d; d >>= 64; }
    }
    if (fe_geq_p(r)) fe_sub_p(r);
}
static void fe_pow(fe *r, const fe *a, const fe *e) {
    fe x = *a, acc = {{1, 0, 0, 0}};
    for (int i = 255; i >= 0; --i) {
        fe_mul(&acc, &acc, &acc);
        if ((e->v[i / 64] >> (i % 64)) & 1) fe_mul(&acc, &acc, &x);
    }
    *r = acc;
}
static void fe_inv(fe *r, const fe *a) { fe e = FP; e.v[0] -= 2; fe_pow(r, a, &e); }
static int fe_is_zero(const fe *a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }
static int fe_eq(const fe *a, const fe *b) { return !memcmp(a, b, sizeof *a); }
static void fe_from(fe *r, const uint8_t b[32]) { for (int i = 0; i < 4; ++i) r->v[i] = be64(b + 8 * (3 - i)); }
static void fe_to(uint8_t b[32], const fe *a) { for (int i = 0; i < 4; ++i) put64(b + 8 * (3 - i), a->v[i]); }

typedef struct { fe X, Y, Z; int inf; } jac;

static void jdbl(jac *r, const jac *p) {
    if (p->inf || fe_is_zero(&p->Y)) { r->inf = 1; return; }
    fe yy, s, m, t, x3, y3, z3;
    fe_mul(&yy, &p->Y, &p->Y);
    fe_mul(&s, &p->X, &yy); fe_add(&s, &s, &s); fe_add(&s, &s, &s);      /* S = 4XY^2 */
    fe_mul(&m, &p->X, &p->X); fe_add(&t, &m, &m); fe_add(&m, &t, &m);   /* M = 3X^2 */
    fe_mul(&x3, &m, &m); fe_sub(&x3, &x3, &s); fe_sub(&x3, &x3, &s);    /* X' = M^2 - 2S */
    fe_mul(&t, &yy, &yy); fe_add(&t, &t, &t); fe_add(&t, &t, &t); fe_add(&t, &t, &t); /* 8Y^4 */
    fe_sub(&y3, &s, &x3); fe_mul(&y3, &m, &y3); fe_sub(&y3, &y3, &t);
    fe_mul(&z3, &p->Y, &p->Z); fe_add(&z3, &z3, &z3);
    r->X = x3; r->Y = y3; r->Z = z3; r->inf = 0;
}

static void jadd(jac *r, const jac *p, const jac *q) {
    if (p->inf) { *r = *q; return; }
    if (q->inf) { *r = *p; return; }
    fe z1z1, z2z2, u1, u2, s1, s2, h, rr_, hh, hhh, v, x3, y3, z3, t;
    fe_mul(&z1z1, &p->Z, &p->Z); fe_mul(&z2z2, &q->Z, &q->Z);
    fe_mul(&u1, &p->X, &z2z2); fe_mul(&u2, &q->X, &z1z1);
    fe_mul(&s1, &p->Y, &q->Z); fe_mul(&s1, &s1, &z2z2);
    fe_mul(&s2, &q->Y, &p->Z); fe_mul(&s2, &s2, &z1z1);
    if (fe_eq(&u1, &u2)) {
        if (fe_eq(&s1, &s2)) { jdbl(r, p); return; }
        r->inf = 1;
        return;
    }
    fe_sub(&h, &u2, &u1); fe_sub(&rr_, &s2, &s1);
    fe_mul(&hh, &h, &h); fe_mul(&hhh, &hh, &h); fe_mul(&v, &u1, &hh);
    fe_mul(&x3, &rr_, &rr_); fe_sub(&x3, &x3, &hhh); fe_sub(&x3, &x3, &v); fe_sub(&x3, &x3, &v);
    fe_sub(&y3, &v, &x3); fe_mul(&y3, &rr_, &y3); fe_mul(&t, &s1, &hhh); fe_sub(&y3, &y3, &t);
    fe_mul(&z3, &p->Z, &q->Z); fe_mul(&z3, &z3, &h);
    r->X = x3; r->Y = y3; r->Z = z3; r->inf = 0;
}

/* affine (x, y) <- k * (px, py); k big-endian 32 bytes */
static int ec_mul(const uint8_t k[32], const fe *px, const fe *py, fe *x, fe *y) {
    jac acc = {.inf = 1}, b = {*px, *py, {{1, 0, 0, 0}}, 0};
    for (int i = 0; i < 256; ++i) {
        jdbl(&acc, &acc);
        if ((k[i / 8] >> (7 - i % 8)) & 1) jadd(&acc, &acc, &b);
    }
    if (acc.inf) return ORC_ERR_ECIES;
    fe zi, z2, z3;
    fe_inv(&zi, &acc.Z);
    fe_mul(&z2, &zi, &zi); fe_mul(&z3, &z2, &zi);
    fe_mul(x, &acc.X, &z2); fe_mul(y, &acc.Y, &z3);
    return ORC_OK;
}

static int valid_scalar(const uint8_t k[32]) {
    int zero = 1;
    for (int i = 0; i < 32; ++i) zero &= k[i] == 0;
    if (zero) return 0;
    for (int i = 0; i < 32; ++i) {
        if (k[i] < ORDER[i]) return 1;
        if (k[i] > ORDER[i]) return 0;
    }
    return 0; /* == n */
}

static int on_curve(const fe *x, const fe *y) {
    fe l, r, seven = {{7, 0, 0, 0}};
    fe_mul(&l, y, y);
    fe_mul(&r, x, x); fe_mul(&r, &r, x); fe_add(&r, &r, &seven);
    return fe_eq(&l, &r);
}

/* PublicKey::parse_slice: 33 (02/03 || x), 64 (x || y) or 65 (04 || x || y) bytes */
static int parse_pub(const uint8_t *pk, uint64_t len, fe *x, fe *y) {
    if (len == 64 || (len == 65 && pk[0] == 4)) {
        const uint8_t *p = len == 64 ? pk : pk + 1;
        fe_from(x, p); fe_from(y, p + 32);
        uint8_t chk[32];
        fe_to(chk, x); if (memcmp(chk, p, 32)) return ORC_ERR_ECIES;       /* coordinate >= p */
        fe_to(chk, y); if (memcmp(chk, p + 32, 32)) return ORC_ERR_ECIES;
    } else if (len == 33 && (pk[0] == 2 || pk[0] == 3)) {
        fe_from(x, pk + 1);
        uint8_t chk[32];
        fe_to(chk, x); if (memcmp(chk, pk + 1, 32)) return ORC_ERR_ECIES;
        fe r, seven = {{7, 0, 0, 0}}, e = FP;
        fe_mul(&r, x, x); fe_mul(&r, &r, x); fe_add(&r, &r, &seven);
        /* sqrt = r^((p+1)/4) */
        u128 c = 1;
        for (int i = 0; i < 4; ++i) { c += e.v[i]; e.v[i] = (uint64_t)c; c >>= 64; }
        for (int i = 0; i < 4; ++i) e.v[i] = (e.v[i] >> 2) | (i < 3 ? e.v[i + 1] << 62 : (uint64_t)c << 62);
        fe_pow(y, &r, &e);
        if ((int)(y->v[0] & 1) != (pk[0] & 1)) { fe z = {{0, 0, 0, 0}}; fe_sub(y, &z, y); }
    } else {
        return ORC_ERR_ECIES;
    }
    return on_curve(x, y) ? ORC_OK : ORC_ERR_ECIES;
}

static void ser65(uint8_t out[65], const fe *x, const fe *y) { out[0] = 4; fe_to(out + 1, x); fe_to(out + 33, y); }

int orc_ecies_public_key(const uint8_t sk[32], uint8_t out[65]) {
    if (!valid_scalar(sk)) return ORC_ERR_ECIES;
    fe gx, gy, x, y;
    fe_from(&gx, GXB); fe_from(&gy, GYB);
    int rc = ec_mul(sk, &gx, &gy, &x, &y);
    if (rc) return rc;
    ser65(out, &x, &y);
    return ORC_OK;
}

/* key = HKDF(eph_pub65 || (peer * k)65) */
static int derive(const uint8_t k[32], const fe *px, const fe *py, const uint8_t eph65[65], uint8_t key[32]) {
    fe sx, sy;
    int rc = ec_mul(k, px, py, &sx, &sy);
    if (rc) return rc;
    uint8_t master[130];
    memcpy(master, eph65, 65);
    ser65(master + 65, &sx, &sy);
    hkdf32(master, 130, key);
    return ORC_OK;
}

int orc_ecies_encrypt(const uint8_t *pub, uint64_t pklen, const uint8_t eph_sk[32], const uint8_t nonce[16],
                      const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if (cap < n + 97) return ORC_ERR_BUFFER_TOO_SMALL;
    fe px, py;
    int rc = parse_pub(pub, pklen, &px, &py);
    if (rc) return rc;
    rc = orc_ecies_public_key(eph_sk, out);
    if (rc) return rc;
    uint8_t key[32];
    rc = derive(eph_sk, &px, &py, out, key);
    if (rc) return rc;
    memcpy(out + 65, nonce, 16);
    gcm(key, nonce, in, n, out + 97, out + 81, 0);
    *out_len = n + 97;
    return ORC_OK;
}

int orc_ecies_decrypt(const uint8_t sk[32], const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                      uint64_t *out_len) {
    if (n < 97 || !valid_scalar(sk)) return ORC_ERR_ECIES;
    if (cap < n - 97) return ORC_ERR_BUFFER_TOO_SMALL;
    fe ex, ey;
    int rc = parse_pub(in, 65, &ex, &ey);
    if (rc) return rc;
    uint8_t key[32], tag[16];
    rc = derive(sk, &ex, &ey, in, key);
    if (rc) return rc;
    memcpy(tag, in + 81, 16);
    rc = gcm(key, in + 65, in + 97, n - 97, out, tag, 1);
    if (rc) return rc;
    *out_len = n - 97;
    return ORC_OK;
}

/* ------------------------------------------------------------ full encode()/decode() */
int orc_encode_full(uint8_t format, const uint8_t *pub, uint64_t pklen, const uint8_t eph_sk[32],
                    const uint8_t nonce[16], const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                    uint64_t *out_len, uint8_t hash[32], orc_encode_info *info) {
    uint8_t *s1 = NULL, *s2 = NULL;
    const uint8_t *cur = in;
    uint64_t cur_n = n, bc = 0, be = 0;
    int rc = ORC_OK;
    if (format & 2) { /* encoding.rs:101-107 */
        s1 = (uint8_t *)malloc(orc_snap_max_len(n) + 1);
        rc = orc_snap_compress(in, n, s1, orc_snap_max_len(n) + 1, &cur_n);
        if (rc) goto done;
        cur = s1;
        bc = cur_n;
    }
    if (format & 1) { /* encoding.rs:109-115 */
        s2 = (uint8_t *)malloc(cur_n + 97);
        rc = orc_ecies_encrypt(pub, pklen, eph_sk, nonce, cur, cur_n, s2, cur_n + 97, &cur_n);
        if (rc) goto done;
        cur = s2;
        be = cur_n;
    }
    rc = orc_encode(format & 12, cur, cur_n, out, cap, out_len, hash, info);
    if (rc) goto done;
    info->input_len = (uint32_t)n;
    info->bytes_compressed = (uint32_t)bc;
    info->bytes_encrypted = (uint32_t)be;
    info->compression_factor = (float)info->bytes_compressed / (float)info->input_len;
    info->amplification_factor = (float)info->bytes_verifiable / (float)info->input_len;
done:
    free(s1);
    free(s2);
    return rc;
}
