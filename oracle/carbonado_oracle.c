/*
 * carbonado_oracle.c — CPU ORACLE (test infrastructure, never the product).
 * See carbonado_oracle.h for scope, citations and parity status.
 *
 * Plain C99, scalar, single-threaded on purpose: it is the checker, and the
 * reference it restates (carbonado 0.6.0 + zfec-rs 0.1.0 + bao 0.12.1) is a
 * single-threaded Rust library.
 */
#include "carbonado_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* GF(2^8), polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2.          */
/* zfec fec.c generate_gf() builds the same tables from Pp="101110001". */
/* ------------------------------------------------------------------ */
static uint8_t gf_exp[512];
static int gf_log[256];
static int gf_ready = 0;

static void gf_init(void) {
    if (gf_ready) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        gf_exp[i] = (uint8_t)x;
        gf_log[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) gf_exp[i] = gf_exp[i - 255];
    gf_log[0] = 255; /* fec.c convention: log(0) is "infinity" */
    gf_ready = 1;
}

/* fec.c keeps a full 256x256 product table (gf_mul_table) for addmul */
static uint8_t gf_mul_table[256][256];
static int gf_table_ready = 0;

static void gf_table_init(void) {
    if (gf_table_ready) return;
    gf_init();
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            gf_mul_table[a][b] = (a && b) ? gf_exp[gf_log[a] + gf_log[b]] : 0;
    gf_table_ready = 1;
}

/* built once at load time, before any thread runs (the checkers call the
   oracle from many threads) */
__attribute__((constructor)) static void gf_tables_at_load(void) { gf_table_init(); }

/* fec.c addmul(dst, src, c, sz): dst[i] ^= c * src[i] by table lookup */
static void addmul(uint8_t *dst, const uint8_t *src, uint8_t c, uint64_t sz) {
    const uint8_t *row = gf_mul_table[c];
    for (uint64_t t = 0; t < sz; t++) dst[t] ^= row[src[t]];
}

uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (!a || !b) return 0;
    return gf_exp[gf_log[a] + gf_log[b]];
}

uint8_t orc_gf_inv(uint8_t a) {
    gf_init();
    if (!a) return 0;
    return gf_exp[255 - gf_log[a]];
}

/* Gauss-Jordan inversion over GF(2^8).  (fec.c uses a Vandermonde-specific
 * inversion for the top block; the inverse is unique, so any exact method
 * yields identical bytes — the Python oracle restates the fec.c route and the
 * tests compare the two.) */
int orc_gf_invert(uint8_t *a, unsigned k) {
    gf_init();
    uint8_t *aug = (uint8_t *)calloc((size_t)k * 2 * k, 1);
    if (!aug) return -1;
    unsigned w = 2 * k;
    for (unsigned r = 0; r < k; r++) {
        memcpy(aug + r * w, a + r * k, k);
        aug[r * w + k + r] = 1;
    }
    for (unsigned c = 0; c < k; c++) {
        unsigned p = c;
        while (p < k && aug[p * w + c] == 0) p++;
        if (p == k) { free(aug); return -1; }
        if (p != c)
            for (unsigned j = 0; j < w; j++) {
                uint8_t t = aug[p * w + j]; aug[p * w + j] = aug[c * w + j]; aug[c * w + j] = t;
            }
        uint8_t iv = orc_gf_inv(aug[c * w + c]);
        for (unsigned j = 0; j < w; j++) aug[c * w + j] = orc_gf_mul(aug[c * w + j], iv);
        for (unsigned r = 0; r < k; r++) {
            if (r == c || aug[r * w + c] == 0) continue;
            uint8_t f = aug[r * w + c];
            for (unsigned j = 0; j < w; j++) aug[r * w + j] ^= orc_gf_mul(f, aug[c * w + j]);
        }
    }
    for (unsigned r = 0; r < k; r++) memcpy(a + r * k, aug + r * w + k, k);
    free(aug);
    return 0;
}

/* fec.c fec_new(k, n): rows of the m x k Vandermonde matrix V are the powers
 * of the evaluation points {0, a^0, a^1, ..., a^(m-2)}:
 *   V[0]   = [1, 0, ..., 0]                 (point 0, with 0^0 = 1)
 *   V[r]   = [a^((r-1)*c mod 255)]_c        (point a^(r-1)), r >= 1
 * enc = V * (V[0..k))^-1, so the top k rows are the identity (systematic). */
int orc_fec_enc_matrix(unsigned k, unsigned m, uint8_t *mat) {
    gf_init();
    if (k < 1 || m < k || m > 256) return ORC_ERR_ZFEC;
    uint8_t *v = (uint8_t *)calloc((size_t)m * k, 1);
    uint8_t *top = (uint8_t *)calloc((size_t)k * k, 1);
    if (!v || !top) { free(v); free(top); return ORC_ERR_ZFEC; }
    v[0] = 1;
    for (unsigned r = 1; r < m; r++)
        for (unsigned c = 0; c < k; c++) v[r * k + c] = gf_exp[((r - 1) * c) % 255];
    memcpy(top, v, (size_t)k * k);
    if (orc_gf_invert(top, k) != 0) { free(v); free(top); return ORC_ERR_ZFEC; }
    for (unsigned r = 0; r < m; r++)
        for (unsigned c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (unsigned t = 0; t < k; t++) acc ^= orc_gf_mul(v[r * k + t], top[t * k + c]);
            mat[r * k + c] = acc;
        }
    free(v);
    free(top);
    return ORC_OK;
}

/* utils.rs:50-58 computes this in f64; restated in integers (exact for all
 * lengths the reference can hold).  target = ceil(n / (1024*k)) * 1024*k. */
void orc_calc_padding_len(uint64_t input_len, unsigned k, uint32_t *padding, uint32_t *chunk_len) {
    uint64_t unit = 1024ull * k;
    uint64_t target = (input_len + unit - 1) / unit * unit;
    *padding = (uint32_t)(target - input_len);
    *chunk_len = (uint32_t)(target / k);
}

/* encoding.rs:48-81: zero-pad to k*chunk_len, split into k contiguous data
 * shards, append m-k parity shards; output is shard-major [S0|S1|...|Sm-1]. */
int orc_zfec_encode(unsigned k, unsigned m, const uint8_t *in, uint64_t n,
                    uint8_t *out, uint64_t out_cap, uint32_t *padding, uint32_t *chunk_len) {
    if (k < 1 || m < k || m > 256) return ORC_ERR_ZFEC;
    uint32_t pad, C;
    orc_calc_padding_len(n, k, &pad, &C);
    uint64_t total = (uint64_t)m * C;
    if (out_cap < total) return ORC_ERR_BUFFER_TOO_SMALL;
    uint8_t *mat = (uint8_t *)malloc((size_t)m * k);
    if (!mat) return ORC_ERR_ZFEC;
    orc_fec_enc_matrix(k, m, mat);
    gf_table_init();
    /* data shards = zero-padded input */
    uint64_t kc = (uint64_t)k * C;
    if (n) memcpy(out, in, n);
    memset(out + n, 0, kc - n);
    for (unsigned i = k; i < m; i++) {
        uint8_t *dst = out + (uint64_t)i * C;
        memset(dst, 0, C);
        for (unsigned j = 0; j < k; j++) {
            uint8_t c = mat[i * k + j];
            if (c) addmul(dst, out + (uint64_t)j * C, c, C);
        }
    }
    free(mat);
    *padding = pad;
    *chunk_len = C;
    return ORC_OK;
}

int orc_zfec_decode_shares(unsigned k, unsigned m, const uint8_t *const *shares,
                           const uint32_t *idx, unsigned nshares, uint64_t chunk_len,
                           uint32_t padding, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (k < 1 || m < k || m > 256) return ORC_ERR_ZFEC;
    uint64_t kc = (uint64_t)k * chunk_len;
    if (padding > kc) return ORC_ERR_ZFEC;
    uint64_t olen = kc - padding;
    if (out_cap < olen) return ORC_ERR_BUFFER_TOO_SMALL;
    /* choose k distinct shares: primaries first (each at its own row), then
     * secondaries in the given order */
    int have[256];
    const uint8_t *sel_ptr[256];
    uint32_t sel_idx[256];
    for (unsigned i = 0; i < 256; i++) have[i] = 0;
    unsigned nsel = 0;
    for (unsigned s = 0; s < nshares; s++) {
        if (idx[s] >= m) return ORC_ERR_ZFEC;
        if (idx[s] < k && !have[idx[s]]) { have[idx[s]] = 1; sel_ptr[nsel] = shares[s]; sel_idx[nsel++] = idx[s]; }
    }
    for (unsigned s = 0; s < nshares && nsel < k; s++)
        if (idx[s] >= k && !have[idx[s]]) { have[idx[s]] = 1; sel_ptr[nsel] = shares[s]; sel_idx[nsel++] = idx[s]; }
    if (nsel < k) return ORC_ERR_ZFEC;
    uint8_t *mat = (uint8_t *)malloc((size_t)m * k);
    uint8_t *dec = (uint8_t *)malloc((size_t)k * k);
    uint8_t *tmp = (uint8_t *)malloc(kc ? kc : 1);
    if (!mat || !dec || !tmp) { free(mat); free(dec); free(tmp); return ORC_ERR_ZFEC; }
    orc_fec_enc_matrix(k, m, mat);
    for (unsigned s = 0; s < k; s++) memcpy(dec + s * k, mat + sel_idx[s] * k, k);
    if (orc_gf_invert(dec, k) != 0) { free(mat); free(dec); free(tmp); return ORC_ERR_ZFEC; }
    for (unsigned r = 0; r < k; r++) {
        uint8_t *dst = tmp + (uint64_t)r * chunk_len;
        if (have[r]) {
            for (unsigned s = 0; s < k; s++)
                if (sel_idx[s] == r) { memcpy(dst, sel_ptr[s], chunk_len); break; }
            continue;
        }
        memset(dst, 0, chunk_len);
        gf_table_init();
        for (unsigned s = 0; s < k; s++) {
            uint8_t c = dec[r * k + s];
            if (c) addmul(dst, sel_ptr[s], c, chunk_len);
        }
    }
    memcpy(out, tmp, olen);
    *out_len = olen;
    free(mat); free(dec); free(tmp);
    return ORC_OK;
}

/* decoding.rs:35-51: len % m must be 0, shards indexed by position 0..m */
int orc_zfec_decode(unsigned k, unsigned m, const uint8_t *in, uint64_t len, uint32_t padding,
                    uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (k < 1 || m < k || m > 256) return ORC_ERR_ZFEC;
    if (len % m != 0) return ORC_ERR_UNEVEN_ZFEC_CHUNKS;
    uint64_t C = len / m;
    const uint8_t *ptrs[256];
    uint32_t idx[256];
    for (unsigned i = 0; i < m; i++) { ptrs[i] = in + i * C; idx[i] = i; }
    return orc_zfec_decode_shares(k, m, ptrs, idx, m, C, padding, out, out_cap, out_len);
}

/* ------------------------------------------------------------------ */
/* BLAKE3 (spec section 2): 7 rounds, SHA-256 IV, message permutation.  */
/* ------------------------------------------------------------------ */
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const unsigned B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static uint32_t rotr(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }

static void g(uint32_t *s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
    s[a] = s[a] + s[b] + x; s[d] = rotr(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + y; s[d] = rotr(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];     s[b] = rotr(s[b] ^ s[c], 7);
}

/* compress -> first 8 words of the output (the chaining value) */
static void compress(const uint32_t cv[8], const uint32_t blk[16], uint64_t counter,
                     uint32_t blen, uint32_t flags, uint32_t out[8]) {
    uint32_t s[16], m[16], t[16];
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    for (int i = 0; i < 4; i++) s[8 + i] = B3_IV[i];
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32); s[14] = blen; s[15] = flags;
    memcpy(m, blk, sizeof m);
    for (int r = 0; r < 7; r++) {
        g(s, 0, 4, 8, 12, m[0], m[1]);  g(s, 1, 5, 9, 13, m[2], m[3]);
        g(s, 2, 6, 10, 14, m[4], m[5]); g(s, 3, 7, 11, 15, m[6], m[7]);
        g(s, 0, 5, 10, 15, m[8], m[9]); g(s, 1, 6, 11, 12, m[10], m[11]);
        g(s, 2, 7, 8, 13, m[12], m[13]); g(s, 3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) out[i] = s[i] ^ s[i + 8];
}

static void load_block(const uint8_t *p, uint32_t len, uint32_t blk[16]) {
    uint8_t b[64];
    memset(b, 0, 64);
    memcpy(b, p, len);
    for (int i = 0; i < 16; i++)
        blk[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 |
                 (uint32_t)b[4 * i + 3] << 24;
}

void orc_blake3_chunk_cv(const uint8_t *chunk, uint32_t len, uint64_t counter, int is_root,
                         uint32_t cv[8]) {
    uint32_t h[8], blk[16];
    memcpy(h, B3_IV, sizeof h);
    uint32_t nblocks = len == 0 ? 1 : (len + 63) / 64;
    for (uint32_t b = 0; b < nblocks; b++) {
        uint32_t blen = (b + 1 == nblocks) ? len - 64 * b : 64;
        uint32_t flags = 0;
        if (b == 0) flags |= CHUNK_START;
        if (b + 1 == nblocks) { flags |= CHUNK_END; if (is_root) flags |= ROOT; }
        load_block(chunk + 64 * b, blen, blk);
        compress(h, blk, counter, blen, flags, h);
    }
    memcpy(cv, h, sizeof h);
}

void orc_blake3_parent_cv(const uint32_t left[8], const uint32_t right[8], int is_root,
                          uint32_t cv[8]) {
    uint32_t blk[16];
    memcpy(blk, left, 32);
    memcpy(blk + 8, right, 32);
    compress(B3_IV, blk, 0, 64, PARENT | (is_root ? ROOT : 0), cv);
}

static void cv_bytes(const uint32_t cv[8], uint8_t out[32]) {
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)cv[i]; out[4 * i + 1] = (uint8_t)(cv[i] >> 8);
        out[4 * i + 2] = (uint8_t)(cv[i] >> 16); out[4 * i + 3] = (uint8_t)(cv[i] >> 24);
    }
}

static void bytes_cv(const uint8_t in[32], uint32_t cv[8]) {
    for (int i = 0; i < 8; i++)
        cv[i] = (uint32_t)in[4 * i] | (uint32_t)in[4 * i + 1] << 8 | (uint32_t)in[4 * i + 2] << 16 |
                (uint32_t)in[4 * i + 3] << 24;
}

/* BLAKE3 tree: the left subtree holds the largest power-of-two number of
 * chunks that leaves at least one byte for the right subtree. */
static uint64_t left_len(uint64_t len) {
    uint64_t full = (len - 1) / 1024;
    uint64_t p = 1;
    while (p * 2 <= full) p *= 2;
    return p * 1024;
}

static void subtree_cv(const uint8_t *in, uint64_t len, uint64_t chunk0, int is_root, uint32_t cv[8]) {
    if (len <= 1024) { orc_blake3_chunk_cv(in, (uint32_t)len, chunk0, is_root, cv); return; }
    uint64_t l = left_len(len);
    uint32_t a[8], b[8];
    subtree_cv(in, l, chunk0, 0, a);
    subtree_cv(in + l, len - l, chunk0 + l / 1024, 0, b);
    orc_blake3_parent_cv(a, b, is_root, cv);
}

void orc_blake3(const uint8_t *in, uint64_t n, uint8_t out[32]) {
    uint32_t cv[8];
    subtree_cv(in, n, 0, 1, cv);
    cv_bytes(cv, out);
}

/* ------------------------------------------------------------------ */
/* bao combined encoding: u64 LE content length, then the tree in      */
/* pre-order (64-byte parent = left CV || right CV, before its subtrees;*/
/* 1 KiB chunks as leaves).                                            */
/* ------------------------------------------------------------------ */
uint64_t orc_bao_encoded_len(uint64_t n) {
    uint64_t chunks = n == 0 ? 1 : (n + 1023) / 1024;
    return 8 + n + 64 * (chunks - 1);
}

static uint64_t bao_enc_rec(const uint8_t *in, uint64_t len, uint64_t chunk0, int is_root,
                            uint8_t *out, uint32_t cv[8]) {
    if (len <= 1024) {
        memcpy(out, in, len);
        orc_blake3_chunk_cv(in, (uint32_t)len, chunk0, is_root, cv);
        return len;
    }
    uint64_t l = left_len(len);
    uint32_t a[8], b[8];
    uint64_t w = 64;
    w += bao_enc_rec(in, l, chunk0, 0, out + w, a);
    w += bao_enc_rec(in + l, len - l, chunk0 + l / 1024, 0, out + w, b);
    cv_bytes(a, out);
    cv_bytes(b, out + 32);
    orc_blake3_parent_cv(a, b, is_root, cv);
    return w;
}

int orc_bao_encode(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint8_t hash[32]) {
    uint64_t need = orc_bao_encoded_len(n);
    if (out_cap < need) return ORC_ERR_BUFFER_TOO_SMALL;
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(n >> (8 * i));
    uint32_t cv[8];
    bao_enc_rec(in, n, 0, 1, out + 8, cv);
    cv_bytes(cv, hash);
    return ORC_OK;
}

/* sequential verifying reader, as bao::decode::decode walks the stream */
typedef struct { const uint8_t *p; uint64_t left; uint8_t *out; uint64_t w; } bao_rd;

static int bao_dec_rec(bao_rd *r, uint64_t len, uint64_t chunk0, int is_root, const uint32_t expect[8]) {
    uint32_t cv[8];
    if (len <= 1024) {
        if (r->left < len) return ORC_ERR_BAO_TRUNCATED;
        orc_blake3_chunk_cv(r->p, (uint32_t)len, chunk0, is_root, cv);
        if (memcmp(cv, expect, 32)) return ORC_ERR_BAO_HASH_MISMATCH;
        memcpy(r->out + r->w, r->p, len);
        r->w += len; r->p += len; r->left -= len;
        return ORC_OK;
    }
    if (r->left < 64) return ORC_ERR_BAO_TRUNCATED;
    uint32_t a[8], b[8];
    bytes_cv(r->p, a);
    bytes_cv(r->p + 32, b);
    orc_blake3_parent_cv(a, b, is_root, cv);
    if (memcmp(cv, expect, 32)) return ORC_ERR_BAO_HASH_MISMATCH;
    r->p += 64; r->left -= 64;
    uint64_t l = left_len(len);
    int rc = bao_dec_rec(r, l, chunk0, 0, a);
    if (rc) return rc;
    return bao_dec_rec(r, len - l, chunk0 + l / 1024, 0, b);
}

int orc_bao_decode(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len,
                   uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (hash_len != 32) return ORC_ERR_HASH_DECODE; /* utils.rs:38-45 */
    if (len < 8) return ORC_ERR_BAO_TRUNCATED;
    uint64_t n = 0;
    for (int i = 0; i < 8; i++) n |= (uint64_t)enc[i] << (8 * i);
    if (orc_bao_encoded_len(n) > len) return ORC_ERR_BAO_TRUNCATED;
    if (out_cap < n) return ORC_ERR_BUFFER_TOO_SMALL;
    uint32_t expect[8];
    bytes_cv(hash, expect);
    bao_rd r = {enc + 8, len - 8, out, 0};
    int rc = bao_dec_rec(&r, n, 0, 1, expect);
    if (rc) return rc;
    *out_len = n;
    return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* encode()/decode() glue for Format bits Bao (4) and Zfec (8).         */
/* constants.rs:49-56: bitmask order Ecies=1, Snappy=2, Bao=4, Zfec=8.  */
/* ------------------------------------------------------------------ */
enum { F_ECIES = 1, F_SNAPPY = 2, F_BAO = 4, F_ZFEC = 8 };

uint64_t orc_encode_max_len(uint64_t n) {
    uint32_t pad, C;
    orc_calc_padding_len(n, 4, &pad, &C);
    uint64_t z = 8ull * C;
    uint64_t b = orc_bao_encoded_len(z > n ? z : n);
    return b > z ? b : z;
}

int orc_encode(uint8_t format, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
               uint64_t *out_len, uint8_t hash[32], orc_encode_info *info) {
    if (format & (F_ECIES | F_SNAPPY)) return ORC_ERR_UNSUPPORTED_FORMAT;
    orc_encode_info inf;
    memset(&inf, 0, sizeof inf);
    inf.input_len = (uint32_t)n;
    const uint8_t *cur = in;
    uint64_t cur_len = n;
    uint8_t *zbuf = NULL;
    if (format & F_ZFEC) { /* encoding.rs:121-130 */
        uint32_t pad, C;
        orc_calc_padding_len(n, 4, &pad, &C);
        zbuf = (uint8_t *)malloc(8ull * C + 1);
        int rc = orc_zfec_encode(4, 8, in, n, zbuf, 8ull * C, &inf.padding_len, &inf.chunk_len);
        if (rc) { free(zbuf); return rc; }
        inf.bytes_ecc = (uint32_t)(8ull * C);
        inf.verifiable_slice_count = (uint16_t)(inf.bytes_ecc / 1024);
        if (inf.verifiable_slice_count % 8 != 0) { free(zbuf); return ORC_ERR_INVALID_VERIFIABLE_SLICE_COUNT; }
        inf.chunk_slice_count = inf.verifiable_slice_count / 8;
        cur = zbuf;
        cur_len = 8ull * C;
    }
    if (format & F_BAO) { /* encoding.rs:140-147 */
        uint64_t need = orc_bao_encoded_len(cur_len);
        if (out_cap < need) { free(zbuf); return ORC_ERR_BUFFER_TOO_SMALL; }
        orc_bao_encode(cur, cur_len, out, out_cap, hash);
        inf.bytes_verifiable = (uint32_t)need;
        cur_len = need;
    } else {
        if (out_cap < cur_len) { free(zbuf); return ORC_ERR_BUFFER_TOO_SMALL; }
        if (cur_len) memcpy(out, cur, cur_len);
        memset(hash, 0, 32);
    }
    free(zbuf);
    inf.compression_factor = (float)inf.bytes_compressed / (float)inf.input_len;
    inf.amplification_factor = (float)inf.bytes_verifiable / (float)inf.input_len;
    inf.output_len = (uint32_t)cur_len;
    *out_len = cur_len;
    if (info) *info = inf;
    return ORC_OK;
}

int orc_decode(const uint8_t *hash, uint64_t hash_len, const uint8_t *in, uint64_t n,
               uint32_t padding, uint8_t format, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (format & (F_ECIES | F_SNAPPY)) return ORC_ERR_UNSUPPORTED_FORMAT;
    uint8_t *vbuf = NULL;
    const uint8_t *cur = in;
    uint64_t cur_len = n;
    if (format & F_BAO) { /* decoding.rs:89-93 */
        if (hash_len != 32) return ORC_ERR_HASH_DECODE;
        vbuf = (uint8_t *)malloc(n + 1);
        uint64_t vl = 0;
        int rc = orc_bao_decode(in, n, hash, hash_len, vbuf, n, &vl);
        if (rc) { free(vbuf); return rc; }
        cur = vbuf;
        cur_len = vl;
    }
    int rc = ORC_OK;
    if (format & F_ZFEC) { /* decoding.rs:95-99 */
        rc = orc_zfec_decode(4, 8, cur, cur_len, padding, out, out_cap, out_len);
    } else {
        if (out_cap < cur_len) rc = ORC_ERR_BUFFER_TOO_SMALL;
        else { if (cur_len) memcpy(out, cur, cur_len); *out_len = cur_len; }
    }
    free(vbuf);
    return rc;
}

/* counter-based generator (SplitMix64 finaliser over a keyed counter) */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_object(uint64_t seed, uint64_t obj, uint8_t *out, uint64_t n) {
    uint64_t key = seed ^ (obj * 0xD1B54A32D192ED03ull);
    for (uint64_t w = 0; w * 8 < n; w++) {
        uint64_t v = mix64(key + (w + 1) * 0x9E3779B97F4A7C15ull);
        for (unsigned b = 0; b < 8 && w * 8 + b < n; b++) out[w * 8 + b] = (uint8_t)(v >> (8 * b));
    }
}
