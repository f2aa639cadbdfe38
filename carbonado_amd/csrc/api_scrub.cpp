// api_scrub.cpp — verify_slice / extract_slice / scrub (decoding.rs:116-212),
// one stream from host memory or a batch of device-resident streams.
// Shared declarations: api_common.hpp.
#include "api_common.hpp"

using namespace chip;
using namespace chip::api;

namespace {

// the one-pass verify of scrub / verify_slice (below): single-object streams
// of up to 4096 chunks (r11zh: at 64 KiB - 1 MiB of content 26-39 % faster
// than the DMA + per-node check, equal at 4 MiB, 9 % slower at 16 MiB)
bool fast_verify_ok(uint64_t n) { return single_ok(n) && n_chunks_of(n) <= 4096; }

// after a failed one-pass verify the stream already sits in the context's
// pinned input (single_decode_km: at byte 64), so the per-node check's upload
// is a direct DMA from there instead of a copy through the staging ring
const uint8_t *pinned_stream(Ctx *c) { return static_cast<const uint8_t *>(c->hin.p) + 64; }

}  // namespace

extern "C" {

// ---- slices and scrub (decoding.rs:116-212) ----------------------------------

uint64_t chip_bao_slice_len(uint64_t n, uint64_t start, uint64_t len) {
    uint64_t c0, c1, total = 8;
    slice_chunks(n, start, len, &c0, &c1);
    std::vector<SliceNode> nodes;
    slice_nodes(n, c0, c1, &nodes);
    for (const SliceNode &sn : nodes) total += sn.len;
    return total;
}

int chip_bao_extract_slice(const uint8_t *enc, uint64_t len, uint64_t index, uint64_t slice_len, uint8_t *out,
                           uint64_t out_cap, uint64_t *out_len) {
    if (!out_len || (!enc && len)) return CHIP_ERR_INVALID_ARG;
    if (index > (~0ull >> 10)) return CHIP_ERR_INVALID_ARG;
    uint64_t n;
    int st = bao_header(enc, len, &n);
    if (st != CHIP_OK) return st;
    uint64_t c0, c1;
    slice_chunks(n, index * 1024, slice_len, &c0, &c1);
    std::vector<SliceNode> nodes;
    slice_nodes(n, c0, c1, &nodes);
    uint64_t total = 8;
    for (const SliceNode &sn : nodes) total += sn.len;
    if (!out || out_cap < total) return CHIP_ERR_BUFFER_TOO_SMALL;
    std::memcpy(out, enc, 8);  // the length header, then the nodes in pre-order
    uint64_t w = 8;
    for (const SliceNode &sn : nodes) {
        std::memcpy(out + w, enc + sn.off, sn.len);
        w += sn.len;
    }
    *out_len = total;
    return CHIP_OK;
}

int chip_bao_verify_slice(const uint8_t *hash, uint64_t hash_len, const uint8_t *enc, uint64_t len,
                          uint64_t index, uint64_t count, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!out_len || (!enc && len)) return CHIP_ERR_INVALID_ARG;
    if (!hash || hash_len != CHIP_HASH_LEN) return CHIP_ERR_HASH_DECODE;
    if (index > (~0ull >> 11) || count > (~0ull >> 11)) return CHIP_ERR_INVALID_ARG;
    uint64_t n;
    int st = bao_header(enc, len, &n);
    if (st != CHIP_OK) return st;
    const uint64_t start = index * 1024, slen = count * 1024;  // decoding.rs:138-139 (u64 maths)
    const uint64_t end = start + slen < n ? start + slen : n;
    const uint64_t olen = start < n ? end - start : 0;
    if (olen && (!out || out_cap < olen)) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    // One verify pass of the whole stream on the single-object path (KM / KS,
    // zero-copy): when every node checks out, so does the slice, and its bytes
    // are the caller's own (gathered here); otherwise the per-node check below
    // decides for this slice alone.  Streams of up to 4096 chunks: beyond, the
    // DMA + per-node check is as fast (r11zh)
    const uint8_t *src = enc;  // the stream the per-node check uploads
    if (fast_verify_ok(n)) {
        st = single_decode_km(c, enc, len, n, hash, nullptr, 0);
        if (st == CHIP_OK) {
            const uint64_t N = n_chunks_of(n);
            for (uint64_t p = start; p < end;) {
                const uint64_t k = p / 1024, o = p % 1024, m = std::min<uint64_t>(1024 - o, end - p);
                std::memcpy(out + (p - start), enc + bao_chunk_offset(k, N) + o, m);
                p += m;
            }
            *out_len = olen;
            return CHIP_OK;
        }
        if (st != CHIP_ERR_BAO_HASH_MISMATCH) return st;
        src = pinned_stream(c);
    }
    const uint64_t blen = bao_encoded_len(n);
    CHIP_HIP(grow(c->in, blen));
    CHIP_HIP(h2d(c->stage, c->in.p, src, blen, c->stream));
    std::vector<uint8_t> cf, pf;
    st = node_check_ctx(c, n, hash, &cf, &pf);
    if (st != CHIP_OK) return st;
    uint64_t c0, c1;
    slice_chunks(n, start, slen, &c0, &c1);
    if (!slice_ok(n, c0, c1, cf, pf)) return CHIP_ERR_BAO_HASH_MISMATCH;
    if (olen) {
        const uint64_t g0 = start / 1024, g1 = (end + 1023) / 1024;
        CHIP_HIP(grow(c->out, (g1 - g0) * 1024));
        CHIP_HIP(bao_gather_content(static_cast<const uint8_t *>(c->in.p), n, g0, g1,
                                    static_cast<uint8_t *>(c->out.p), c->stream));
        CHIP_HIP(d2h(c->stage, out, static_cast<uint8_t *>(c->out.p) + (start - g0 * 1024), olen, c->stream));
        CHIP_HIP(small_sync(c));
    }
    *out_len = olen;
    return CHIP_OK;
}

int chip_scrub(const uint8_t *enc, uint64_t len, const uint8_t *hash, uint64_t hash_len, uint32_t padding,
               uint32_t chunk_len, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!out_len || (!enc && len)) return CHIP_ERR_INVALID_ARG;
    if (!hash || hash_len != CHIP_HASH_LEN) return CHIP_ERR_HASH_DECODE;  // decoding.rs:164
    uint64_t n;
    int st = bao_header(enc, len, &n);
    if (st != CHIP_OK) return st;
    Ctx *c;
    st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    // A healthy stream (periodic scrubbing's usual case, decoding.rs:151-158)
    // is answered by one verify pass of the whole stream on the single-object
    // path (KM / KS, zero-copy); a damaged one takes the per-node check and
    // the repair below (paying that pass too: ~115 us at 1 MiB of content).
    const uint8_t *src = enc;  // the stream the per-node check uploads
    if (fast_verify_ok(n)) {
        st = single_decode_km(c, enc, len, n, hash, nullptr, 0);
        if (st == CHIP_OK) return CHIP_ERR_UNNECESSARY_SCRUB;  // decoding.rs:169-170
        if (st != CHIP_ERR_BAO_HASH_MISMATCH) return st;
        src = pinned_stream(c);
    }
    const uint64_t blen = bao_encoded_len(n);
    CHIP_HIP(grow(c->in, blen));
    CHIP_HIP(h2d(c->stage, c->in.p, src, blen, c->stream));
    std::vector<uint8_t> cf, pf;
    st = node_check_ctx(c, n, hash, &cf, &pf);
    if (st != CHIP_OK) return st;
    bool all = true;
    for (uint8_t f : cf) all &= f != 0;
    for (uint8_t f : pf) all &= f != 0;
    if (all) return CHIP_ERR_UNNECESSARY_SCRUB;  // decoding.rs:169-170
    const uint64_t C = chunk_len;
    if (C == 0 || C % 1024 || n != (uint64_t)CHIP_FEC_M * C) return CHIP_ERR_ZFEC;
    const uint64_t spc = C / 1024;  // slices per chunk, decoding.rs:166
    std::vector<uint32_t> good;
    for (uint32_t i = 0; i < CHIP_FEC_M; ++i)  // decoding.rs:173-183
        if (slice_ok(n, i * spc, (i + 1) * spc, cf, pf)) good.push_back(i);
    CHIP_HIP(grow(c->out, len));
    CHIP_HIP(grow(c->small, 64));
    uint8_t *d_h2 = static_cast<uint8_t *>(c->small.p);
    st = scrub_repair_enqueue(c, static_cast<const uint8_t *>(c->in.p), n, len, good, padding, C,
                              static_cast<uint8_t *>(c->out.p), d_h2);
    if (st != CHIP_OK) return st;
    uint8_t h2[32];
    CHIP_HIP(small_d2h(c, h2, d_h2, 32));
    CHIP_HIP(small_sync(c));
    if (std::memcmp(h2, hash, 32) != 0) return CHIP_ERR_INVALID_SCRUBBED_HASH;  // decoding.rs:205-207
    if (!out || out_cap < len) return CHIP_ERR_BUFFER_TOO_SMALL;
    CHIP_HIP(d2h(c->stage, out, c->out.p, len, c->stream));
    CHIP_HIP(small_sync(c));
    *out_len = len;
    return CHIP_OK;
}

// damaged streams repaired per batch (scratch: ~5 x the stream per object)
constexpr size_t kScrubGroup = 64;

uint64_t chip_scrub_scratch_len(uint64_t len, uint64_t count) {
    uint64_t n = 0;
    if (!bao_content_len(len, &n)) return 16;
    const uint64_t N = n_chunks_of(n);
    return ((count * (2 * N - 1) + count + 15) & ~uint64_t(15)) + 16;
}

int chip_scrub_batch_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t len, uint64_t count,
                         const uint8_t *d_hash, uint32_t padding, uint32_t chunk_len, uint8_t *d_out,
                         uint64_t out_stride, int32_t *status, void *d_scratch, void *stream) {
    if (count == 0) return CHIP_OK;
    if (!d_in || !d_hash || !d_out || !status || !d_scratch) return CHIP_ERR_INVALID_ARG;
    uint64_t n = 0;
    if (!bao_content_len(len, &n) || in_stride < len || out_stride < len) return CHIP_ERR_INVALID_ARG;
    // streams at any 8-B phase (56 mod 64: every chunk and node on a 64-B
    // boundary): the check kernels read them in 8-B units or aligned lines,
    // the gather with 8-B aligned loads, and repaired rows land by a copy
    if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out) | in_stride | out_stride) % 8)
        return CHIP_ERR_INVALID_ARG;
    const uint64_t C = chunk_len;
    if (C == 0 || C % 1024 || n != (uint64_t)CHIP_FEC_M * C) return CHIP_ERR_ZFEC;
    int st = use_device();
    if (st != CHIP_OK) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t N = n_chunks_of(n);
    uint8_t *cf = static_cast<uint8_t *>(d_scratch), *pf = cf + count * N, *masks = pf + count * (N - 1);
    // every node of every stream, then each stream's authentic shards (decoding.rs:168-183)
    CHIP_HIP(bao_node_check(d_in, in_stride, n, count, d_hash, cf, pf, s));
    CHIP_HIP(scrub_masks(d_in, in_stride, n, count, C / 1024, cf, pf, masks, s));
    std::vector<uint8_t> m(count), want(32 * count);
    CHIP_HIP(hipMemcpyAsync(m.data(), masks, count, hipMemcpyDeviceToHost, s));
    CHIP_HIP(hipMemcpyAsync(want.data(), d_hash, 32 * count, hipMemcpyDeviceToHost, s));
    CHIP_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> repair;
    for (uint64_t o = 0; o < count; ++o) {
        const int good = __builtin_popcount(m[o]);
        if (good == CHIP_FEC_M) status[o] = CHIP_ERR_UNNECESSARY_SCRUB;  // decoding.rs:169-170
        else if (good < CHIP_FEC_K) status[o] = CHIP_ERR_ZFEC;          // zfec_chunks: too few shares
        else repair.push_back(o);
    }
    if (repair.empty()) return CHIP_OK;
    // the damaged streams in groups of up to kScrubGroup, as batches: gather
    // each stream's content, zfec decode per share pattern (the group sorted
    // by pattern), one fused re-encode of the group, rows copied to d_out;
    // one synchronisation per group.  (One object at a time, each launch ran
    // nearly empty: ~0.19 ms per 16 MiB object.)
    Ctx *c;
    st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    const uint64_t kc = (uint64_t)CHIP_FEC_K * C;
    struct Rep { uint64_t o; std::vector<uint32_t> sel; };
    std::vector<Rep> reps;
    uint32_t pad2 = 0;
    uint64_t C2 = 0;
    const bool pad_ok = padding <= kc;
    if (pad_ok) calc_pad(kc - padding, CHIP_FEC_K, &pad2, &C2);
    for (uint64_t o : repair) {  // the host-side verdicts, as scrub_repair_enqueue's order
        std::vector<uint32_t> good, pos;
        for (uint32_t i = 0; i < CHIP_FEC_M; ++i)
            if (m[o] >> i & 1) good.push_back(i);
        if (!pad_ok) { status[o] = CHIP_ERR_ZFEC; continue; }
        if (pad2 != padding) { status[o] = CHIP_ERR_SCRUBBED_PADDING_MISMATCH; continue; }
        if (bao_encoded_len((uint64_t)CHIP_FEC_M * C2) != len) { status[o] = CHIP_ERR_SCRUBBED_LENGTH_MISMATCH; continue; }
        if (select_shares(CHIP_FEC_K, CHIP_FEC_M, good.data(), (uint32_t)good.size(), &pos) != CHIP_OK) {
            status[o] = CHIP_ERR_ZFEC;
            continue;
        }
        Rep r{o, {}};
        for (uint32_t p : pos) r.sel.push_back(good[p]);
        reps.push_back(std::move(r));
    }
    std::stable_sort(reps.begin(), reps.end(), [](const Rep &a, const Rep &b) { return a.sel < b.sel; });
    const uint64_t z2 = (uint64_t)CHIP_FEC_M * C2, lstride = (len + 15) & ~uint64_t(15);
    for (size_t g0 = 0; g0 < reps.size(); g0 += kScrubGroup) {
        const size_t R = std::min(kScrubGroup, reps.size() - g0);
        CHIP_HIP(grow(c->mid, R * n));
        CHIP_HIP(grow(c->x1, R * kc));
        CHIP_HIP(grow(c->x2, R * lstride));
        CHIP_HIP(grow(c->flags, 32 * R));
        CHIP_HIP(grow(c->scratch, std::max(zfec_bao_scratch_len(z2, R), bao_scratch_len(z2, R))));
        uint8_t *d_z = static_cast<uint8_t *>(c->mid.p), *d_dec = static_cast<uint8_t *>(c->x1.p);
        uint8_t *d_enc = static_cast<uint8_t *>(c->x2.p), *d_h2 = static_cast<uint8_t *>(c->flags.p);
        for (size_t j = 0; j < R; ++j)
            CHIP_HIP(bao_gather_content(d_in + reps[g0 + j].o * in_stride, n, 0, N, d_z + j * n, c->stream));
        for (size_t j = 0; j < R;) {  // zfec decode from the authentic shares, TRUE indices (decoding.rs:187)
            size_t e2 = j + 1;
            while (e2 < R && reps[g0 + e2].sel == reps[g0 + j].sel) ++e2;
            std::vector<uint64_t> slot_off(CHIP_FEC_K);
            for (uint32_t k2 = 0; k2 < CHIP_FEC_K; ++k2) slot_off[k2] = reps[g0 + j].sel[k2] * C;
            st = zfec_decode_device(CHIP_FEC_K, CHIP_FEC_M, d_z + j * n, n, slot_off, reps[g0 + j].sel, C, e2 - j,
                                    d_dec + j * kc, kc, c->stream);
            if (st != CHIP_OK) return st;
            j = e2;
        }
        // re-encode (decoding.rs:191-196): encode() at Zfec|Bao of every decoded object, one fused pass
        CHIP_HIP(zfec_bao_dev(d_dec, kc, kc - padding, R, C2, d_enc, lstride, d_h2, c->scratch.p, c->stream));
        std::vector<uint8_t> h2(32 * R);
        CHIP_HIP(small_d2h(c, h2.data(), d_h2, h2.size()));
        CHIP_HIP(small_sync(c));
        for (size_t j = 0; j < R; ++j) {  // decoding.rs:205-207
            const uint64_t o = reps[g0 + j].o;
            const bool ok = std::memcmp(h2.data() + 32 * j, want.data() + 32 * o, 32) == 0;
            status[o] = ok ? CHIP_OK : CHIP_ERR_INVALID_SCRUBBED_HASH;
            // only a repaired stream whose hash matches is handed out, as
            // chip_scrub (the next group's work is behind these copies on the
            // same stream)
            if (ok)
                CHIP_HIP(hipMemcpyAsync(d_out + o * out_stride, d_enc + j * lstride, len, hipMemcpyDeviceToDevice,
                                        c->stream));
        }
    }
    CHIP_HIP(hipStreamSynchronize(c->stream));
    return CHIP_OK;
}

}  // extern "C"
