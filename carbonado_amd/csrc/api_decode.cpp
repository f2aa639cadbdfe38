// api_decode.cpp — decode() from host memory (decoding.rs:80-114): one
// object (chip_decode) and the pipelined host batch (chip_decode_host_batch:
// H2D, bao verify-decode, D2H, host stages on host threads).  Shared
// declarations: api_common.hpp.
#include <condition_variable>
#include <mutex>
#include <thread>

#include "api_common.hpp"

using namespace chip;
using namespace chip::api;

namespace {

// device-stage geometry of one encoded object (decoding.rs:80-99)
struct DecGeom {
    int st = CHIP_OK;
    uint64_t blen = 0;  // bytes entering zfec (bao content length, or the input length)
    uint64_t olen = 0;  // bytes leaving zfec (k*C - padding, or blen)
};

// decode()'s host stages (decoding.rs:101-111) on the device stages' output
// cur[0, cur_n): ECIES (with the key derived ahead, when there is one) then
// snappy, or the two in one pass; a large object on the stage pool.
int host_tail(const uint8_t *secret_key, uint64_t sk_len, bool ecies, bool snap, const uint8_t *cur, uint64_t cur_n,
              uint8_t *out, uint64_t out_cap, uint64_t *out_len, const uint8_t *pre_key, const uint8_t *pre_eph) {
    Trace trace("host stages");
    struct Mark {
        Trace &t;
        ~Mark() { t.mark("decode"); }
    } mark{trace};
    if (ecies && snap)  // decoding.rs:101-111 in one pass
        return host::ecies_decrypt_snap_par(secret_key, sk_len, cur, cur_n, out, out_cap, out_len, pre_key, pre_eph);
    if (ecies) {  // decoding.rs:101-105
        uint64_t got = 0;
        const int st = host::ecies_decrypt_par(secret_key, sk_len, cur, cur_n, out, out_cap, &got, pre_key, pre_eph);
        if (st == CHIP_OK || st == CHIP_ERR_BUFFER_TOO_SMALL) *out_len = got;
        return st;
    }
    return host::snap_decompress_par(cur, cur_n, out, out_cap, out_len);  // decoding.rs:107-111
}

// CHIP_DEC_SPEC=0: a decode's host stages wait for the device's verdict
// instead of running on the unverified content meanwhile (an A/B knob)
bool dec_spec_on() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_DEC_SPEC");
        return !(e && e[0] == '0');
    }();
    return on;
}

DecGeom dec_geom(uint8_t format, const uint8_t *in, uint64_t n, uint32_t padding) {
    DecGeom g;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    g.blen = n;
    if (bao) {
        g.st = bao_header(in, n, &g.blen);
        if (g.st != CHIP_OK) return g;
    }
    g.olen = g.blen;
    if (zfec) {
        if (g.blen % CHIP_FEC_M) { g.st = CHIP_ERR_UNEVEN_ZFEC_CHUNKS; return g; }  // decoding.rs:39-41
        const uint64_t C = g.blen / CHIP_FEC_M;
        if (padding > CHIP_FEC_K * C) { g.st = CHIP_ERR_ZFEC; return g; }
        g.olen = CHIP_FEC_K * C - padding;
    }
    return g;
}

}  // namespace

extern "C" {

int chip_decode_host_batch(uint8_t format, const uint8_t *secret_key, uint64_t sk_len, const uint8_t *hashes,
                           const uint8_t *in, const uint64_t *in_len, uint64_t count, uint64_t in_stride,
                           const uint32_t *padding, uint8_t *out, uint64_t out_stride, uint64_t *out_len,
                           int32_t *status, uint32_t nslots, uint64_t slice_bytes, uint32_t host_threads) {
    if (count == 0) return CHIP_OK;
    if (!in || !in_len || !out_len || !status || !padding) return CHIP_ERR_INVALID_ARG;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    const bool hs = has_host_stages(format);
    if ((format & CHIP_FORMAT_ECIES) && !secret_key) return CHIP_ERR_INVALID_ARG;
    if (bao && !hashes) return CHIP_ERR_HASH_DECODE;
    // host-side geometry and the largest sizes
    std::vector<DecGeom> geo(count);
    uint64_t in_max = 0, mid_max = 0, olen_max = 0;
    for (uint64_t o = 0; o < count; ++o) {
        geo[o] = dec_geom(format, in + o * in_stride, in_len[o], padding[o]);
        status[o] = geo[o].st;
        in_max = std::max(in_max, in_len[o]);
        mid_max = std::max(mid_max, geo[o].blen);
        olen_max = std::max(olen_max, geo[o].olen);
    }
    if (!zfec && !bao) {  // host stages only (or identity)
        for (uint64_t o = 0; o < count; ++o) {
            if (status[o] != CHIP_OK) continue;
            const uint8_t *src = in + o * in_stride;
            uint64_t n = in_len[o];
            uint8_t *dst = out + o * out_stride;
            if (!hs) {
                if (n > out_stride && count > 1) { status[o] = CHIP_ERR_BUFFER_TOO_SMALL; out_len[o] = n; continue; }
                std::memcpy(dst, src, n);
                out_len[o] = n;
                continue;
            }
            uint64_t got = 0;
            int st = CHIP_OK;
            if ((format & CHIP_FORMAT_ECIES) && (format & CHIP_FORMAT_SNAPPY)) {
                st = host::ecies_decrypt_snap_par(secret_key, sk_len, src, n, dst, out_stride, &got);
            } else if (format & CHIP_FORMAT_ECIES) {  // Ecies alone here (Ecies|Snappy above)
                st = host::ecies_decrypt_par(secret_key, sk_len, src, n, dst, out_stride, &got);
            }
            else if (format & CHIP_FORMAT_SNAPPY) st = host::snap_decompress(src, n, dst, out_stride, &got);
            status[o] = st;
            out_len[o] = got;
        }
        for (uint64_t o = 0; o < count; ++o)
            if (status[o] != CHIP_OK) return status[o];
        return CHIP_OK;
    }
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    nslots = nslots < 1 ? 3 : (nslots > 8 ? 8 : nslots);
    if (slice_bytes == 0) slice_bytes = 256ull << 20;
    uint32_t T = host_threads ? host_threads : std::max(1u, std::thread::hardware_concurrency());
    T = std::min<uint32_t>(T, 64);
    const uint64_t i_al = row_pitch(in_max), m_al = row_pitch(mid_max), o_al = (olen_max + 15) / 16 * 16;
    uint64_t S = slice_bytes / (in_max ? in_max : 1);
    S = S < 1 ? 1 : (S > count ? count : S);
    if (c->slots.size() < nslots) c->slots.resize(nslots);
    for (uint32_t k = 0; k < nslots; ++k) {
        Slot &sl = c->slots[k];
        if (!sl.stream) CHIP_HIP(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
        CHIP_HIP(grow(sl.in, S * i_al));
        if (bao) {
            CHIP_HIP(grow(sl.mid, S * m_al));
            CHIP_HIP(grow(sl.scratch, bao_scratch_len(mid_max, S)));
            CHIP_HIP(grow(sl.hash, S * 32 + S * 4));  // hashes, then per-object status words
        }
        if (hs) CHIP_HIP(grow_pinned(sl.stage, S * o_al + S * 4));
        else if (bao) CHIP_HIP(grow_pinned(sl.stage, S * 4));
    }
    const uint64_t nslices = (count + S - 1) / S;
    std::vector<Scratch> dscratch(T);  // per host thread, reused across slices
    // host part of slice i: device statuses -> status[], then ecies -> snap into out
    auto finish = [&](uint64_t i) {
        Slot &sl = c->slots[i % nslots];
        const uint64_t o0 = i * S, cnt = std::min(S, count - o0);
        const uint8_t *stage = static_cast<const uint8_t *>(sl.stage.p);
        const uint32_t *dst_st = reinterpret_cast<const uint32_t *>(stage + (hs ? S * o_al : 0));
        for (uint64_t j = 0; j < cnt; ++j)
            if (bao && status[o0 + j] == CHIP_OK && dst_st[j]) status[o0 + j] = (int32_t)dst_st[j];
        if (!hs) return;
        const uint32_t nt = (uint32_t)std::min<uint64_t>(T, cnt);
        auto work = [&](uint32_t t) {
            Scratch &tmp = dscratch[t];
            for (uint64_t j = t; j < cnt; j += nt) {
                const uint64_t o = o0 + j;
                if (status[o] != CHIP_OK) continue;
                const uint8_t *src = stage + j * o_al;
                uint64_t n = geo[o].olen, got = 0;
                uint8_t *dst = out + o * out_stride;
                int r = CHIP_OK;
                if ((format & CHIP_FORMAT_ECIES) && (format & CHIP_FORMAT_SNAPPY)) {  // one pass, no plaintext buffer
                    status[o] = host::ecies_decrypt_snap(secret_key, sk_len, src, n, dst, out_stride, &got,
                                                         tmp.get(host::DECRYPT_SNAP_WINDOW));
                    out_len[o] = got;
                    continue;
                }
                if (format & CHIP_FORMAT_ECIES) {
                    const bool snap = format & CHIP_FORMAT_SNAPPY;
                    uint8_t *tb = snap ? tmp.get(n + 1) : nullptr;
                    r = host::ecies_decrypt(secret_key, sk_len, src, n, snap ? tb : dst, snap ? n + 1 : out_stride,
                                            &got);
                    src = tb;
                    n = got;
                }
                if (r == CHIP_OK && (format & CHIP_FORMAT_SNAPPY)) r = host::snap_decompress(src, n, dst, out_stride, &got);
                status[o] = r;
                out_len[o] = got;
            }
        };
        std::vector<std::thread> pool;
        for (uint32_t t = 1; t < nt; ++t) pool.emplace_back(work, t);
        work(0);
        for (auto &th : pool) th.join();
    };
    // device part of slice i (H2D, bao verify, D2H) enqueued on its slot's stream
    auto enqueue = [&](uint64_t i) -> int {
        Slot &sl = c->slots[i % nslots];
        const uint64_t o0 = i * S, cnt = std::min(S, count - o0);
        uint8_t *stage = static_cast<uint8_t *>(sl.stage.p);
        uint32_t *h_st = reinterpret_cast<uint32_t *>(stage + (hs ? S * o_al : 0));
        for (uint64_t j = 0; j < cnt; ++j) { h_st[j] = 0; if (!hs) out_len[o0 + j] = geo[o0 + j].olen; }
        // uniform slice -> one batched pass; otherwise object by object
        bool uniform = true;
        for (uint64_t j = 1; j < cnt; ++j)
            uniform &= in_len[o0 + j] == in_len[o0] && geo[o0 + j].blen == geo[o0].blen &&
                       geo[o0 + j].olen == geo[o0].olen;
        for (uint64_t j = 0; j < cnt; ++j) uniform &= geo[o0 + j].st == CHIP_OK;
        const uint64_t groups = uniform ? 1 : cnt;
        for (uint64_t gI = 0; gI < groups; ++gI) {
            const uint64_t j0 = uniform ? 0 : gI, gcnt = uniform ? cnt : 1, o = o0 + j0;
            if (geo[o].st != CHIP_OK) continue;
            const uint64_t n = in_len[o], blen = geo[o].blen, olen = geo[o].olen;
            uint8_t *d_in = static_cast<uint8_t *>(sl.in.p) + j0 * i_al;
            if (n) CHIP_HIP(hipMemcpy2DAsync(d_in, i_al, in + o * in_stride, count > 1 ? in_stride : n, n, gcnt,
                                             hipMemcpyHostToDevice, sl.stream));
            const uint8_t *d_res = d_in;
            uint64_t res_pitch = i_al;
            if (bao) {  // decoding.rs:89-93, all objects of the group verified in one pass
                uint8_t *d_hash = static_cast<uint8_t *>(sl.hash.p) + j0 * 32;
                uint32_t *d_st = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(sl.hash.p) + S * 32) + j0;
                CHIP_HIP(hipMemcpyAsync(d_hash, hashes + 32 * o, 32 * gcnt, hipMemcpyHostToDevice, sl.stream));
                CHIP_HIP(hipMemsetAsync(d_st, 0, 4 * gcnt, sl.stream));
                uint8_t *d_mid = static_cast<uint8_t *>(sl.mid.p) + j0 * m_al;
                // every byte verified; only the bytes zfec keeps (the data shards) written
                // (CHIP_DECODE_PREFIX=0: round 4's whole-content verify-decode, the A/B of DESIGN §6)
                static const bool prefix = env_int("CHIP_DECODE_PREFIX", 1) != 0;
                if (prefix)
                    CHIP_HIP(bao_decode_prefix_dev(d_in, i_al, blen, gcnt, d_hash, d_mid, m_al, zfec ? olen : blen,
                                                   d_st, sl.scratch.p, sl.stream));
                else
                    CHIP_HIP(bao_decode_dev(d_in, i_al, blen, gcnt, d_hash, d_mid, m_al, d_st, sl.scratch.p,
                                            sl.stream));
                CHIP_HIP(hipMemcpyAsync(h_st + j0, d_st, 4 * gcnt, hipMemcpyDeviceToHost, sl.stream));
                d_res = d_mid;
                res_pitch = m_al;
            }
            // zfec (decoding.rs:95-99): the shards are indexed by position, so the
            // primaries are present and decode = their bytes, padding dropped
            if (olen) {
                uint8_t *dst = hs ? stage + j0 * o_al : out + o * out_stride;
                const uint64_t dpitch = hs ? o_al : (count > 1 ? out_stride : olen);
                if (!hs && count > 1 && olen > out_stride) {
                    for (uint64_t j = 0; j < gcnt; ++j) status[o + j] = CHIP_ERR_BUFFER_TOO_SMALL;
                    continue;
                }
                CHIP_HIP(hipMemcpy2DAsync(dst, dpitch, d_res, res_pitch, olen, gcnt, hipMemcpyDeviceToHost, sl.stream));
            }
        }
        return CHIP_OK;
    };
    // A finisher thread completes slices in order (wait for the slot's stream,
    // then the host stages on T threads) while this thread keeps the device
    // queue full; a slot is reused only after its previous slice finished.
    std::mutex fm;
    std::condition_variable fcv;
    uint64_t enqueued = 0, finished = 0;
    bool abort_run = false;
    std::string fin_err;
    std::thread finisher([&] {
        (void)hipSetDevice(c->dev);
        for (uint64_t i = 0; i < nslices; ++i) {
            {
                std::unique_lock<std::mutex> lk(fm);
                fcv.wait(lk, [&] { return enqueued > i || abort_run; });
                if (enqueued <= i) return;
            }
            hipError_t e = hipStreamSynchronize(c->slots[i % nslots].stream);
            if (e == hipSuccess) finish(i);
            std::lock_guard<std::mutex> lk(fm);
            if (e != hipSuccess) {
                fin_err = hipGetErrorString(e);
                abort_run = true;
            }
            finished = i + 1;
            fcv.notify_all();
            if (abort_run) return;
        }
    });
    int run_st = CHIP_OK;
    for (uint64_t i = 0; i < nslices && run_st == CHIP_OK; ++i) {
        if (i >= nslots) {
            std::unique_lock<std::mutex> lk(fm);
            fcv.wait(lk, [&] { return finished > i - nslots || abort_run; });
            if (abort_run) { run_st = CHIP_ERR_DEVICE; break; }
        }
        run_st = enqueue(i);
        std::lock_guard<std::mutex> lk(fm);
        if (run_st == CHIP_OK) enqueued = i + 1;
        else abort_run = true;
        fcv.notify_all();
    }
    finisher.join();
    if (!fin_err.empty()) {
        t_last_err = fin_err;
        run_st = CHIP_ERR_DEVICE;
    }
    if (run_st != CHIP_OK) {
        for (uint32_t k = 0; k < nslots; ++k) (void)hipStreamSynchronize(c->slots[k].stream);
        return run_st;
    }
    for (uint32_t k = 0; k < nslots; ++k) CHIP_HIP(hipStreamSynchronize(c->slots[k].stream));
    for (uint64_t o = 0; o < count; ++o)
        if (status[o] != CHIP_OK) return status[o];
    return CHIP_OK;
}

int chip_decode(const uint8_t *secret_key, uint64_t sk_len, const uint8_t *hash, uint64_t hash_len,
                const uint8_t *in, uint64_t n, uint32_t padding, uint8_t format, uint8_t *out, uint64_t out_cap,
                uint64_t *out_len) {
    if ((!in && n) || !out_len) return CHIP_ERR_INVALID_ARG;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    const bool ecies = format & CHIP_FORMAT_ECIES, snap = format & CHIP_FORMAT_SNAPPY;
    if (ecies && !secret_key) return CHIP_ERR_INVALID_ARG;
    // device stages write to `out` directly unless host stages follow
    thread_local std::vector<uint8_t> t_dev;
    const uint8_t *cur = in;
    uint64_t cur_n = n;
    uint8_t pre_eph[65], pre_key[32];  // ECIES key derived while the device works
    bool have_pre = false;
    struct Wipe {
        uint8_t *k;
        ~Wipe() { host::secure_wipe(k, 32); }
    } wipe_pre{pre_key};
    if (zfec || bao) {
        uint64_t blen = n;
        if (bao) {
            if (!hash || hash_len != CHIP_HASH_LEN) return CHIP_ERR_HASH_DECODE;
            int st = bao_header(in, n, &blen);
            if (st != CHIP_OK) return st;
        }
        uint64_t C = 0, olen = blen;
        if (zfec) {
            if (blen % CHIP_FEC_M != 0) return CHIP_ERR_UNEVEN_ZFEC_CHUNKS;  // decoding.rs:39-41
            C = blen / CHIP_FEC_M;
            if (padding > CHIP_FEC_K * C) return CHIP_ERR_ZFEC;
            if (C % 16) return CHIP_ERR_ZFEC;
            olen = CHIP_FEC_K * C - padding;
        }
        uint8_t *dst = out;
        if (ecies || snap) {
            t_dev.resize(olen + 1);
            dst = t_dev.data();
        } else if (olen && (!out || out_cap < olen)) {
            *out_len = olen;
            return CHIP_ERR_BUFFER_TOO_SMALL;
        }
        Ctx *c;
        int st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        if (bao && single_ok(blen)) {  // KM / KS verifies; the host gathers [0, olen) from `in` meanwhile
            // (at Bao|Zfec the positional shares' primaries are the content's first 4 C bytes)
            // while the device verifies, also the ECIES key from the envelope header as `in` holds it
            auto prekey = [&] {
                if (!ecies) return;
                const uint64_t h0 = bao_chunk_offset(0, (blen + 1023) / 1024);
                if (h0 + 65 <= n && blen >= 65) {
                    std::memcpy(pre_eph, in + h0, 65);
                    have_pre = host::ecies_derive_key(secret_key, sk_len, pre_eph, pre_key) == CHIP_OK;
                }
            };
            // and then the host stages themselves on the gathered (still unverified) content,
            // into `out`: released only with the device's verdict, wiped without it
            int spec = -1;
            const uint64_t out_len0 = *out_len;
            auto stages = [&] {
                if (!(ecies || snap) || !dec_spec_on() || (ecies && !have_pre)) return;
                spec = host_tail(secret_key, sk_len, ecies, snap, dst, olen, out, out_cap, out_len, pre_key, pre_eph);
            };
            st = single_decode_km(c, in, n, blen, hash, dst, olen, prekey, stages);
            if (spec >= 0) {
                if (st == CHIP_OK) return spec;
                if (out && out_cap) host::secure_wipe(out, spec == CHIP_OK ? *out_len : out_cap);
                *out_len = out_len0;
            }
            if (st != CHIP_OK) return st;
            cur = dst;
            cur_n = olen;
        } else if (zfec && !bao && C && zc_ok(2 * CHIP_FEC_K * C)) {  // decoding.rs:95-99: shards by position
            // zero-copy: the decode kernel reads the four primaries from pinned memory
            auto prekey = [&] {
                if (!ecies || n < 65) return;
                std::memcpy(pre_eph, in, 65);
                have_pre = host::ecies_derive_key(secret_key, sk_len, pre_eph, pre_key) == CHIP_OK;
            };
            const uint8_t *sh[CHIP_FEC_K];
            std::vector<uint32_t> sel(CHIP_FEC_K);
            for (uint32_t s = 0; s < CHIP_FEC_K; ++s) { sh[s] = in + s * C; sel[s] = s; }
            st = single_zfec_decode_zc(c, CHIP_FEC_K, CHIP_FEC_M, sh, sel, C, dst, olen, prekey);
            if (st != CHIP_OK) return st;
            cur = dst;
            cur_n = olen;
        } else {
            const uint64_t in_bytes = bao ? bao_encoded_len(blen) : n;
            CHIP_HIP(grow(c->in, in_bytes));
            if (in_bytes) CHIP_HIP(h2d(c->stage, c->in.p, in, in_bytes, c->stream));
            const uint8_t *d_cur = static_cast<const uint8_t *>(c->in.p);
            uint32_t verdict = 0;  // bao's, read at the synchronisation below
            if (bao && zfec) {  // decoding.rs:89-99: the positional shares' primaries are the content's
                // first 4 C bytes, so zfec's decode is the prefix: verify all, write olen bytes
                CHIP_HIP(grow(c->mid, olen));
                st = bao_decode_ctx(c, d_cur, in_bytes, blen, hash, static_cast<uint8_t *>(c->mid.p), olen, &verdict);
                if (st != CHIP_OK) return st;
                d_cur = static_cast<const uint8_t *>(c->mid.p);
            } else if (bao) {  // decoding.rs:89-93
                CHIP_HIP(grow(c->mid, blen));
                st = bao_decode_ctx(c, d_cur, in_bytes, blen, hash, static_cast<uint8_t *>(c->mid.p), ~0ull, &verdict);
                if (st != CHIP_OK) return st;
                d_cur = static_cast<const uint8_t *>(c->mid.p);
            }
            if (zfec && !bao && C) {  // decoding.rs:95-99: shards by position, primaries present
                CHIP_HIP(grow(c->out, CHIP_FEC_K * C));
                std::vector<uint32_t> sel(CHIP_FEC_K);
                std::vector<uint64_t> slot_off(CHIP_FEC_K);
                for (uint32_t s = 0; s < CHIP_FEC_K; ++s) { sel[s] = s; slot_off[s] = s * C; }
                st = zfec_decode_device(CHIP_FEC_K, CHIP_FEC_M, d_cur, 0, slot_off, sel, C, 1,
                                        static_cast<uint8_t *>(c->out.p), 0, c->stream);
                if (st != CHIP_OK) return st;
                d_cur = static_cast<const uint8_t *>(c->out.p);
            }
            // While the device verifies: the ECIES key from the envelope header as the
            // input holds it (content bytes [0, 65): chunk 0 of the bao stream, or the
            // first shard); decrypt uses it only if the verified header is the same
            // (the pool path and the one-thread paths alike, so it is never paid twice)
            if (ecies) {
                const uint64_t h0 = bao ? bao_chunk_offset(0, (blen + 1023) / 1024) : 0;
                if (h0 + 65 <= n && (!bao || blen >= 65)) {
                    std::memcpy(pre_eph, in + h0, 65);
                    have_pre = host::ecies_derive_key(secret_key, sk_len, pre_eph, pre_key) == CHIP_OK;
                }
            }
            if (olen) CHIP_HIP(d2h(c->stage, dst, d_cur, olen, c->stream));
            CHIP_HIP(small_sync(c));
            if (verdict) {  // never hand back unverified content
                if (olen) std::memset(dst, 0, olen);
                return (int)verdict;
            }
            cur = dst;
            cur_n = olen;
        }
    }
    if (!ecies && !snap) {
        if (!(zfec || bao)) {
            if (n && (!out || out_cap < n)) {
                *out_len = n;
                return CHIP_ERR_BUFFER_TOO_SMALL;
            }
            if (n) std::memcpy(out, in, n);
        }
        *out_len = cur_n;
        return CHIP_OK;
    }
    return host_tail(secret_key, sk_len, ecies, snap, cur, cur_n, out, out_cap, out_len, have_pre ? pre_key : nullptr,
                     pre_eph);
}

}  // extern "C"
