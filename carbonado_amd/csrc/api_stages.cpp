// api_stages.cpp — the stage functions the reference routes its hot path
// through (encoding::{zfec, bao}, decoding::{zfec, zfec_chunks, bao},
// encoding.rs:38-81, decoding.rs:21-60), the host stages (snap, ecies), and
// the device-resident batch entry points the throughput is measured on.
// Shared declarations: api_common.hpp.
#include "api_common.hpp"

using namespace chip;
using namespace chip::api;

extern "C" {

// ---- host stages --------------------------------------------------------

int chip_snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if ((!in && n) || !out_len || (n && !out)) return CHIP_ERR_INVALID_ARG;
    return host::snap_compress_par(in, n, out, out_cap, out_len);  // (a large input's blocks on the stage pool)
}

int chip_snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if ((!in && n) || !out_len) return CHIP_ERR_INVALID_ARG;
    return host::snap_decompress_par(in, n, out, out_cap, out_len);
}

int chip_ecies_encrypt(const uint8_t *pubkey, uint64_t pubkey_len, const chip_ecies_inject *inject,
                       const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!pubkey || (!in && n) || !out || !out_len) return CHIP_ERR_INVALID_ARG;
    // a large message's AES-GCM on the stage pool (same bytes; small ones, or a busy pool, on this thread)
    advise_huge(out, std::min(out_cap, n + host::ECIES_OVERHEAD));
    return host::ecies_encrypt_par_plain(pubkey, pubkey_len, inject ? inject->ephemeral_sk : nullptr,
                                         inject ? inject->nonce : nullptr, in, n, out, out_cap, out_len);
}

int chip_ecies_decrypt(const uint8_t *secret_key, uint64_t sk_len, const uint8_t *in, uint64_t n, uint8_t *out,
                       uint64_t out_cap, uint64_t *out_len) {
    if (!secret_key || (!in && n) || !out_len) return CHIP_ERR_INVALID_ARG;
    if (out) advise_huge(out, std::min(out_cap, n));
    return host::ecies_decrypt_par(secret_key, sk_len, in, n, out, out_cap, out_len);
}

int chip_ecies_public_key(const uint8_t *secret_key, uint8_t pubkey[65]) {
    if (!secret_key || !pubkey) return CHIP_ERR_INVALID_ARG;
    return host::ecies_public_key(secret_key, pubkey);
}


// ---- zfec --------------------------------------------------------------

int chip_zfec_encode_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                               uint64_t n, uint64_t count, uint8_t *d_out, uint64_t out_stride,
                               void *stream) {
    if (!valid_km(k, m)) return CHIP_ERR_ZFEC;
    if ((!d_in && n) || !d_out || (in_stride % 16) || (out_stride % 16) || misaligned16(d_in) ||
        misaligned16(d_out))
        return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    uint32_t pad;
    uint64_t C;
    calc_pad(n, k, &pad, &C);
    if (count > 1 && out_stride < (uint64_t)m * C) return CHIP_ERR_INVALID_ARG;
    if (count > 1 && d_in != d_out && in_stride < n) return CHIP_ERR_INVALID_ARG;  // rows would overlap
    // in place (SURVEY 8d "aliased"): data shards are the input bytes themselves
    const bool aliased = d_in == d_out && n;
    if (aliased && count > 1 && in_stride != out_stride) return CHIP_ERR_INVALID_ARG;
    GfPlan p = encode_plan(k, m, C, zfec_enc_matrix(k, m), aliased);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (aliased && (uint64_t)k * C > n)  // the zero padding of encoding.rs:53-55 becomes part of shard k-1
        CHIP_HIP(hipMemset2DAsync(d_out + n, out_stride ? out_stride : (uint64_t)m * C, 0, (uint64_t)k * C - n,
                                  count, s));
    CHIP_HIP(zf_run(count, s, [&](uint64_t o0, uint64_t cnt, hipStream_t st) {
        GfLaunch L{d_in + o0 * in_stride, d_out + o0 * out_stride, in_stride, out_stride, n, C, cnt};
        return gf_apply(p, L, st);
    }));
    return CHIP_OK;
}

int chip_hbm_pattern_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride, uint64_t n,
                               uint64_t count, uint8_t *d_out, uint64_t out_stride, void *stream) {
    if (!((k == 4 && m == 8) || (k == 8 && m == 16))) return CHIP_ERR_ZFEC;
    if ((!d_in && n) || !d_out || d_in == d_out || (in_stride % 16) || (out_stride % 16) || misaligned16(d_in) ||
        misaligned16(d_out))
        return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    uint32_t pad;
    uint64_t C;
    calc_pad(n, k, &pad, &C);
    if (count > 1 && (out_stride < (uint64_t)m * C || in_stride < n)) return CHIP_ERR_INVALID_ARG;
    GfPlan p = encode_plan(k, m, C, zfec_enc_matrix(k, m), false);
    CHIP_HIP(zf_run(count, static_cast<hipStream_t>(stream), [&](uint64_t o0, uint64_t cnt, hipStream_t s) {
        GfLaunch L{d_in + o0 * in_stride, d_out + o0 * out_stride, in_stride, out_stride, n, C, cnt};
        L.pattern_only = true;
        return gf_apply(p, L, s);
    }));
    return CHIP_OK;
}

int chip_zfec_encode(uint32_t k, uint32_t m, const uint8_t *in, uint64_t n, uint8_t *out,
                     uint64_t out_cap, uint32_t *padding, uint32_t *chunk_len) {
    if (!valid_km(k, m)) return CHIP_ERR_ZFEC;
    if ((!in && n) || !padding || !chunk_len) return CHIP_ERR_INVALID_ARG;
    uint32_t pad;
    uint64_t C;
    calc_pad(n, k, &pad, &C);
    const uint64_t total = (uint64_t)m * C;
    if (total && (!out || out_cap < total)) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    if (n && k == 4 && m == 8 && zc_ok(total)) {  // one 4-of-8 object: zero-copy parity, data shards by the host
        st = single_zfec_encode_zc(c, in, n, C, out);
        if (st != CHIP_OK) return st;
    } else if (n) {
        CHIP_HIP(grow(c->in, n));
        CHIP_HIP(grow(c->out, total));
        CHIP_HIP(h2d(c->stage, c->in.p, in, n, c->stream));
        GfPlan p = encode_plan(k, m, C, zfec_enc_matrix(k, m));
        GfLaunch L{static_cast<const uint8_t *>(c->in.p), static_cast<uint8_t *>(c->out.p), 0, 0, n, C, 1};
        CHIP_HIP(gf_apply(p, L, c->stream));
        CHIP_HIP(d2h(c->stage, out, c->out.p, total, c->stream));
        CHIP_HIP(small_sync(c));
    }
    *padding = pad;
    *chunk_len = (uint32_t)C;
    return CHIP_OK;
}

int chip_zfec_decode_shares(uint32_t k, uint32_t m, const uint8_t *const *shares,
                            const uint32_t *idx, uint32_t nshares, uint64_t chunk_len,
                            uint32_t padding, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!valid_km(k, m)) return CHIP_ERR_ZFEC;
    if (!shares || !idx || !out_len) return CHIP_ERR_INVALID_ARG;
    const uint64_t kc = (uint64_t)k * chunk_len;
    if (padding > kc) return CHIP_ERR_ZFEC;
    if (chunk_len % 16) return CHIP_ERR_ZFEC;  // carbonado shards are multiples of 1 KiB
    std::vector<uint32_t> pos;
    int st = select_shares(k, m, idx, nshares, &pos);
    if (st != CHIP_OK) return st;
    const uint64_t olen = kc - padding;
    if (olen && (!out || out_cap < olen)) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    if (kc && zc_ok(2 * kc)) {  // one object: zero-copy (the kernel reads and writes pinned memory)
        std::vector<uint32_t> sel(k);
        std::vector<const uint8_t *> src(k);
        for (uint32_t s = 0; s < k; ++s) { sel[s] = idx[pos[s]]; src[s] = shares[pos[s]]; }
        st = single_zfec_decode_zc(c, k, m, src.data(), sel, chunk_len, out, olen);
        if (st != CHIP_OK) return st;
    } else if (kc) {
        CHIP_HIP(grow(c->in, kc));
        CHIP_HIP(grow(c->out, kc));
        std::vector<uint32_t> sel(k);
        std::vector<uint64_t> slot_off(k);
        for (uint32_t s = 0; s < k; ++s) {
            sel[s] = idx[pos[s]];
            slot_off[s] = (uint64_t)s * chunk_len;
            CHIP_HIP(h2d(c->stage, static_cast<uint8_t *>(c->in.p) + slot_off[s], shares[pos[s]], chunk_len,
                         c->stream));
        }
        st = zfec_decode_device(k, m, static_cast<const uint8_t *>(c->in.p), 0, slot_off, sel, chunk_len,
                                1, static_cast<uint8_t *>(c->out.p), 0, c->stream);
        if (st != CHIP_OK) return st;
        if (olen) CHIP_HIP(d2h(c->stage, out, c->out.p, olen, c->stream));
        CHIP_HIP(small_sync(c));
    }
    *out_len = olen;
    return CHIP_OK;
}

int chip_zfec_decode(uint32_t k, uint32_t m, const uint8_t *in, uint64_t len, uint32_t padding,
                     uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!valid_km(k, m)) return CHIP_ERR_ZFEC;
    if ((!in && len) || !out_len) return CHIP_ERR_INVALID_ARG;
    if (len % m != 0) return CHIP_ERR_UNEVEN_ZFEC_CHUNKS;  // decoding.rs:39-41
    const uint64_t C = len / m;
    std::vector<const uint8_t *> ptrs(m);
    std::vector<uint32_t> idx(m);
    for (uint32_t i = 0; i < m; ++i) { ptrs[i] = in + i * C; idx[i] = i; }  // decoding.rs:24-25
    return chip_zfec_decode_shares(k, m, ptrs.data(), idx.data(), m, C, padding, out, out_cap, out_len);
}

int chip_zfec_decode_batch_dev(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                               uint64_t chunk_len, const uint32_t *idx, uint32_t nshares,
                               uint64_t count, uint8_t *d_out, uint64_t out_stride, void *stream) {
    if (!valid_km(k, m)) return CHIP_ERR_ZFEC;
    if (!d_in || !d_out || !idx || (in_stride % 16) || (out_stride % 16) || (chunk_len % 16) ||
        misaligned16(d_in) || misaligned16(d_out))
        return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    std::vector<uint32_t> pos;
    st = select_shares(k, m, idx, nshares, &pos);
    if (st != CHIP_OK) return st;
    std::vector<uint32_t> sel(k);
    std::vector<uint64_t> slot_off(k);
    uint64_t row_in = 0;
    for (uint32_t s = 0; s < k; ++s) {
        sel[s] = idx[pos[s]];
        slot_off[s] = (uint64_t)sel[s] * chunk_len;
        row_in = std::max(row_in, slot_off[s] + chunk_len);
    }
    // rows would overlap
    if (count > 1 && (in_stride < row_in || out_stride < (uint64_t)k * chunk_len)) return CHIP_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    int part_st = CHIP_OK;
    const hipError_t e = zf_run(count, s, [&](uint64_t o0, uint64_t cnt, hipStream_t st) {
        const int r = zfec_decode_device(k, m, d_in + o0 * in_stride, in_stride, slot_off, sel, chunk_len, cnt,
                                         d_out + o0 * out_stride, out_stride, st);
        if (r != CHIP_OK) part_st = r;
        return r == CHIP_OK ? hipSuccess : hipErrorInvalidValue;
    });
    if (part_st != CHIP_OK) return part_st;
    CHIP_HIP(e);
    return CHIP_OK;
}


int chip_bao_encode_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash,
                              void *d_scratch, void *stream) {
    if ((!d_in && n) || !d_hash || !d_scratch) return CHIP_ERR_INVALID_ARG;
    if (count > 1 && (in_stride < n || (d_out && out_stride < bao_encoded_len(n)))) return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    CHIP_HIP(bao_encode_dev(d_in, in_stride, n, count, d_out, out_stride, d_hash, d_scratch,
                            static_cast<hipStream_t>(stream)));
    return CHIP_OK;
}

int chip_bao_decode_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                              const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride,
                              uint32_t *d_status, void *d_scratch, void *stream) {
    if (!d_in || !d_hash || !d_status || !d_scratch || (!d_out && n)) return CHIP_ERR_INVALID_ARG;
    if (count > 1 && (in_stride < bao_encoded_len(n) || out_stride < n)) return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    CHIP_HIP(hipMemsetAsync(d_status, 0, count * sizeof(uint32_t), s));
    CHIP_HIP(bao_decode_dev(d_in, in_stride, n, count, d_hash, d_out, out_stride, d_status, d_scratch, s));
    return CHIP_OK;
}

uint64_t chip_encode_scratch_len(uint8_t format, uint64_t n, uint64_t count) {
    chip_encode_info inf;
    uint64_t zlen, fl;
    if (encode_info_for(format, n, n, 0, 0, &inf, &zlen, &fl) != CHIP_OK) return 16;
    if ((format & CHIP_FORMAT_BAO) && (format & CHIP_FORMAT_ZFEC))  // fused K13: level-0 CVs of every chunk
        return std::max(zfec_bao_scratch_len(zlen, count), bao_scratch_len(zlen, count)) + 16;
    return (format & CHIP_FORMAT_BAO) ? bao_scratch_len(zlen, count) + 16 : 16;
}

int chip_encode_batch_dev(uint8_t format, const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                          uint8_t *d_out, uint64_t out_stride, uint64_t *out_len, uint8_t *d_hash,
                          chip_encode_info *info, void *d_scratch, void *stream) {
    if (has_host_stages(format) || format > 15) return CHIP_ERR_INVALID_ARG;
    if ((!d_in && n) || !out_len || (!d_hash && count) || (in_stride % 16) || misaligned16(d_in))
        return CHIP_ERR_INVALID_ARG;
    chip_encode_info inf;
    uint64_t zlen, fl;
    int st = encode_info_for(format, n, n, 0, 0, &inf, &zlen, &fl);
    if (st != CHIP_OK) return st;
    {  // output rows: 16-B aligned, or 8-B aligned where K13 writes the streams
        const bool bao8 = (format & CHIP_FORMAT_BAO) && zlen;
        const bool any8 = bao8 && ((format & CHIP_FORMAT_ZFEC) ? zfec_bao_any8(inf.chunk_len, count)
                                                                : (zlen + 1023) / 1024 > KS_MAX_N);
        const uint64_t a = any8 ? 8 : 16;
        if ((out_stride % a) || (reinterpret_cast<uintptr_t>(d_out) % a)) return CHIP_ERR_INVALID_ARG;
    }
    if ((fl && !d_out) || (count > 1 && out_stride < fl)) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (count > 1 && in_stride < n) return CHIP_ERR_INVALID_ARG;  // rows would overlap
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    if (bao && !d_scratch) return CHIP_ERR_INVALID_ARG;
    *out_len = fl;
    if (info) *info = inf;
    if (count == 0) return CHIP_OK;
    st = use_device();
    if (st != CHIP_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (zfec && bao && zlen) {
        CHIP_HIP(zfec_bao_dev(d_in, in_stride, n, count, inf.chunk_len, d_out, out_stride, d_hash, d_scratch, s));
    } else if (zfec) {
        if (zlen) {
            const GfPlan p = encode_plan(CHIP_FEC_K, CHIP_FEC_M, inf.chunk_len, zfec_enc_matrix(CHIP_FEC_K, CHIP_FEC_M));
            GfLaunch L{d_in, d_out, in_stride, out_stride, n, inf.chunk_len, count};
            CHIP_HIP(gf_apply(p, L, s));
        }
        if (bao)  // empty input: bao of the empty zfec output
            CHIP_HIP(bao_encode_dev(d_in, in_stride, 0, count, d_out, out_stride, d_hash, d_scratch, s));
        else
            CHIP_HIP(hipMemsetAsync(d_hash, 0, 32 * count, s));
    } else if (bao) {
        CHIP_HIP(bao_encode_dev(d_in, in_stride, n, count, d_out, out_stride, d_hash, d_scratch, s));
    } else {  // no device stage: the encoding is the input
        if (n) CHIP_HIP(copy_rows_dev(d_out, count > 1 ? out_stride : n, d_in, count > 1 ? in_stride : n, n, count, s));
        CHIP_HIP(hipMemsetAsync(d_hash, 0, 32 * count, s));
    }
    return CHIP_OK;
}

uint64_t chip_decode_scratch_len(uint8_t format, uint64_t in_len, uint64_t count) {
    uint64_t n = 0;
    if (!(format & CHIP_FORMAT_BAO) || !bao_content_len(in_len, &n)) return 16;
    return bao_scratch_len(n, count) + 16;
}

int chip_decode_batch_dev(uint8_t format, const uint8_t *d_in, uint64_t in_stride, uint64_t in_len, uint64_t count,
                          const uint8_t *d_hash, uint32_t padding, uint8_t *d_out, uint64_t out_stride,
                          uint64_t *out_len, uint32_t *d_status, void *d_scratch, void *stream) {
    if (has_host_stages(format) || format > 15 || !out_len) return CHIP_ERR_INVALID_ARG;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    if ((!d_in && in_len) || (count && !d_status) || (out_stride % 16) || misaligned16(d_out))
        return CHIP_ERR_INVALID_ARG;
    uint64_t blen = in_len;  // bytes entering zfec (decoding.rs:90-99)
    {  // input rows: 16-B aligned, or 8-B aligned streams where K3 reads them (over 512 chunks)
        uint64_t cl = 0;
        const bool in8 = bao && bao_content_len(in_len, &cl) && !small_ok(cl, count);
        const uint64_t a = in8 ? 8 : 16;
        if ((in_stride % a) || (reinterpret_cast<uintptr_t>(d_in) % a)) return CHIP_ERR_INVALID_ARG;
    }
    if (bao && !d_hash) return CHIP_ERR_HASH_DECODE;
    if (bao && !d_scratch) return CHIP_ERR_INVALID_ARG;
    if (bao && !bao_content_len(in_len, &blen)) return CHIP_ERR_BAO_TRUNCATED;
    uint64_t olen = blen;
    if (zfec) {
        if (blen % CHIP_FEC_M) return CHIP_ERR_UNEVEN_ZFEC_CHUNKS;  // decoding.rs:39-41
        const uint64_t C = blen / CHIP_FEC_M;
        if (padding > CHIP_FEC_K * C) return CHIP_ERR_ZFEC;
        olen = CHIP_FEC_K * C - padding;  // positional shards: the primaries' bytes (decoding.rs:24-29)
    }
    *out_len = olen;
    if (count == 0) return CHIP_OK;
    if ((olen && !d_out) || (count > 1 && out_stride < olen)) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (count > 1 && in_stride < in_len) return CHIP_ERR_INVALID_ARG;  // rows would overlap
    int st = use_device();
    if (st != CHIP_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    CHIP_HIP(hipMemsetAsync(d_status, 0, count * sizeof(uint32_t), s));
    if (bao) {  // every node verified; only content bytes [0, olen) written
        CHIP_HIP(bao_decode_prefix_dev(d_in, in_stride, blen, count, d_hash, d_out, out_stride, olen, d_status,
                                       d_scratch, s));
    } else if (olen) {
        CHIP_HIP(copy_rows_dev(d_out, count > 1 ? out_stride : olen, d_in, count > 1 ? in_stride : olen, olen, count,
                               s));
    }
    return CHIP_OK;
}

int chip_bao_encode(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                    uint8_t hash[CHIP_HASH_LEN]) {
    if ((!in && n) || !hash || !out_len) return CHIP_ERR_INVALID_ARG;
    const uint64_t blen = bao_encoded_len(n);
    if (!out || out_cap < blen) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    if (single_ok(n)) {  // one object on KM (or KS), zero-copy: only the nodes come back from KM
        st = single_encode_km(c, in, n, 0, blen, out, hash);
        if (st != CHIP_OK) return st;
        *out_len = blen;
        return CHIP_OK;
    }
    CHIP_HIP(grow(c->in, n));
    if (n) CHIP_HIP(h2d(c->stage, c->in.p, in, n, c->stream));
    st = bao_encode_ctx(c, static_cast<const uint8_t *>(c->in.p), n, true, hash);
    if (st != CHIP_OK) return st;
    CHIP_HIP(d2h(c->stage, out, c->out.p, blen, c->stream));
    CHIP_HIP(small_sync(c));
    *out_len = blen;
    return CHIP_OK;
}

int chip_blake3(const uint8_t *in, uint64_t n, uint8_t hash[CHIP_HASH_LEN]) {
    if ((!in && n) || !hash) return CHIP_ERR_INVALID_ARG;
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    CHIP_HIP(grow(c->in, n));
    if (n) CHIP_HIP(h2d(c->stage, c->in.p, in, n, c->stream));
    st = bao_encode_ctx(c, static_cast<const uint8_t *>(c->in.p), n, false, hash);
    if (st != CHIP_OK) return st;
    CHIP_HIP(small_sync(c));
    return CHIP_OK;
}

int chip_bao_decode(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len,
                    uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!out_len || (!enc && len)) return CHIP_ERR_INVALID_ARG;
    if (!hash || hash_len != CHIP_HASH_LEN) return CHIP_ERR_HASH_DECODE;  // utils.rs:38-45
    uint64_t n;
    int st = bao_header(enc, len, &n);
    if (st != CHIP_OK) return st;
    if (n && (!out || out_cap < n)) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    if (single_ok(n)) {  // KM (or KS) verifies on the device while the host gathers the content from `enc`
        st = single_decode_km(c, enc, len, n, hash, out, n);
        if (st != CHIP_OK) return st;
        *out_len = n;
        return CHIP_OK;
    }
    const uint64_t blen = bao_encoded_len(n);
    CHIP_HIP(grow(c->in, blen));
    CHIP_HIP(grow(c->out, n));
    CHIP_HIP(h2d(c->stage, c->in.p, enc, blen, c->stream));
    uint32_t verdict = 0;
    st = bao_decode_ctx(c, static_cast<const uint8_t *>(c->in.p), blen, n, hash,
                        static_cast<uint8_t *>(c->out.p), ~0ull, &verdict);
    if (st != CHIP_OK) return st;
    if (n) CHIP_HIP(d2h(c->stage, out, c->out.p, n, c->stream));
    CHIP_HIP(small_sync(c));
    if (verdict) {  // never hand back unverified content
        if (n) std::memset(out, 0, n);
        return (int)verdict;
    }
    *out_len = n;
    return CHIP_OK;
}

}  // extern "C"
