// api_encode.cpp — encode() from host memory (encoding.rs:86-172): one
// object (chip_encode) and the pipelined host batch (chip_encode_host_batch:
// host stages on host threads, H2D, K13, split copy-back).  Shared
// declarations: api_common.hpp.
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>

#include "api_common.hpp"

using namespace chip;
using namespace chip::api;

extern "C" {

// ---- pipeline glue -------------------------------------------------------

int chip_encode(uint8_t format, const uint8_t *pubkey, uint64_t pubkey_len, const chip_ecies_inject *inject,
                const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len,
                uint8_t hash[CHIP_HASH_LEN], chip_encode_info *info) {
    if ((!in && n) || !out_len || !hash) return CHIP_ERR_INVALID_ARG;
    if ((format & CHIP_FORMAT_ECIES) && !pubkey) return CHIP_ERR_INVALID_ARG;
    // host stages (encoding.rs:101-115)
    thread_local std::vector<uint8_t> t_stage;
    thread_local Scratch t_tmp;
    const uint8_t *cur = in;
    uint64_t cur_n = n, bc = 0, be = 0;
    if (has_host_stages(format)) {
        Trace trace("host stages");
        // straight into the context's pinned input when a device stage follows
        // (the single-object paths then read it there, the others DMA it from
        // there): no copy of the staged bytes into pinned memory afterwards
        const uint64_t cap = host_stage_max(format, n) + 1;
        uint8_t *dst = nullptr;
        Ctx *c = nullptr;
        if ((format & (CHIP_FORMAT_ZFEC | CHIP_FORMAT_BAO)) && zc_ok(cap + 16) && ctx_get(&c) == CHIP_OK &&
            grow_pinned_local(c->hin, cap + 16) == hipSuccess)
            dst = static_cast<uint8_t *>(c->hin.p);
        if (!dst) {
            t_stage.resize(cap);
            dst = t_stage.data();
        }
        int st = host_stages_into(format, pubkey, pubkey_len, inject ? inject->ephemeral_sk : nullptr,
                                  inject ? inject->nonce : nullptr, in, n, dst, cap, t_tmp, &cur_n, &bc, &be, nullptr,
                                  nullptr, nullptr, true);
        if (st != CHIP_OK) return st;
        cur = dst;
        trace.mark("encode");
    }
    chip_encode_info inf;
    uint64_t cur_len, final_len;
    int st = encode_info_for(format, n, cur_n, bc, be, &inf, &cur_len, &final_len);
    if (st != CHIP_OK) return st;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    if (final_len && (!out || out_cap < final_len)) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (!zfec && !bao) {
        if (cur_n) std::memcpy(out, cur, cur_n);
        std::memset(hash, 0, 32);
    } else if (bao && single_ok(cur_len)) {  // one object on KM (split copy-back) or KS, zero-copy (api_single.cpp)
        Ctx *c;
        st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        st = single_encode_km(c, cur, cur_n, zfec ? inf.chunk_len : 0, final_len, out, hash);
        if (st != CHIP_OK) return st;
    } else if (zfec && !bao && cur_n && zc_ok((uint64_t)CHIP_FEC_M * inf.chunk_len)) {  // encoding.rs:121-138 alone: zero-copy parity
        Ctx *c;
        st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        st = single_zfec_encode_zc(c, cur, cur_n, inf.chunk_len, out);
        if (st != CHIP_OK) return st;
        std::memset(hash, 0, 32);  // encoding.rs:145
    } else {
        Ctx *c;
        st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        CHIP_HIP(grow(c->in, cur_n));
        if (cur_n) CHIP_HIP(h2d(c->stage, c->in.p, cur, cur_n, c->stream));
        const uint8_t *d_cur = static_cast<const uint8_t *>(c->in.p);
        if (zfec && bao && cur_len) {  // fused: shards written into the bao stream, hashed in place
            CHIP_HIP(grow(c->out, final_len));
            CHIP_HIP(grow(c->scratch, std::max(zfec_bao_scratch_len(cur_len, 1), bao_scratch_len(cur_len, 1))));
            CHIP_HIP(grow(c->small, 64));
            uint8_t *d_hash = static_cast<uint8_t *>(c->small.p);
            CHIP_HIP(zfec_bao_dev(d_cur, 0, cur_n, 1, inf.chunk_len, static_cast<uint8_t *>(c->out.p), 0, d_hash,
                                  c->scratch.p, c->stream));
            CHIP_HIP(small_d2h(c, hash, d_hash, 32));
            CHIP_HIP(d2h(c->stage, out, c->out.p, final_len, c->stream));
            CHIP_HIP(small_sync(c));
            *out_len = final_len;
            if (info) *info = inf;
            return CHIP_OK;
        }
        if (zfec && cur_len) {
            CHIP_HIP(grow(c->mid, cur_len));
            GfPlan p = encode_plan(CHIP_FEC_K, CHIP_FEC_M, inf.chunk_len, zfec_enc_matrix(CHIP_FEC_K, CHIP_FEC_M));
            GfLaunch L{d_cur, static_cast<uint8_t *>(c->mid.p), 0, 0, cur_n, inf.chunk_len, 1};
            CHIP_HIP(gf_apply(p, L, c->stream));
            d_cur = static_cast<const uint8_t *>(c->mid.p);
        }
        if (bao) {  // encoding.rs:140-142: the zfec output stays on the device
            st = bao_encode_ctx(c, d_cur, cur_len, true, hash);
            if (st != CHIP_OK) return st;
            CHIP_HIP(d2h(c->stage, out, c->out.p, final_len, c->stream));
        } else {
            std::memset(hash, 0, 32);  // encoding.rs:145
            if (final_len) CHIP_HIP(d2h(c->stage, out, d_cur, final_len, c->stream));
        }
        CHIP_HIP(small_sync(c));
    }
    *out_len = final_len;
    if (info) *info = inf;
    return CHIP_OK;
}

namespace {

// encode() at Zfec|Bao from host memory, split copy-back: the stream's data
// region [0, t0) -- its header, the data-shard chunks [0, nd) and the parent
// nodes between them -- is half of the stream, and all of it but the nodes
// is the zero-padded input the host already holds.  The host writes the
// header and those chunks itself (host::fill_data_chunks, while it stages the
// slice); the device gathers the region's nodes into a compact buffer
// (bao_data_nodes); only that buffer and the tail [t0, final) cross PCIe,
// and the host scatters the nodes into their slots once the slot's stream
// is done.  D2H per 16 MiB object: 18.9 MB instead of 35.7.
// CHIP_E2E_SPLIT=0: copy the whole stream back.
struct SplitGeo {
    uint64_t N = 0, nd = 0, t0 = 0, nb = 0;  // chunks, data chunks, data-region end, its nodes
    std::vector<uint64_t> coff;              // [nd] stream offsets of the data chunks
    struct Run {
        uint64_t dst, src, len;  // stream offset, offset in the compact buffer, bytes
    };
    std::vector<Run> runs;
    static SplitGeo make(uint64_t N) {
        SplitGeo g;
        g.N = N;
        g.nd = N / 2;  // 4 of the 8 shards
        g.coff.resize(g.nd);
        uint64_t prev_end = 8, src = 0;
        for (uint64_t i = 0; i < g.nd; ++i) {
            g.coff[i] = bao_chunk_offset(i, N);
            if (g.coff[i] > prev_end) {
                g.runs.push_back({prev_end, src, g.coff[i] - prev_end});
                src += g.coff[i] - prev_end;
            }
            prev_end = g.coff[i] + 1024;
        }
        g.t0 = prev_end;
        g.nb = src / 64;
        return g;
    }
};

// CHIP_E2E_DIRECT=0: Ecies objects go through the pinned staging rows
bool direct_rows_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_E2E_DIRECT");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

bool e2e_split_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_E2E_SPLIT");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

// per-call cache of the geometry by chunk count (objects of a call may differ)
struct SplitGeos {
    std::mutex mu;
    std::map<uint64_t, SplitGeo> by_n;
    const SplitGeo &get(uint64_t N) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = by_n.find(N);
        if (it == by_n.end()) it = by_n.emplace(N, SplitGeo::make(N)).first;
        return it->second;
    }
};

// chunk count of the bao stream of a Zfec|Bao object whose host stages left len bytes
uint64_t split_chunks(uint64_t len) {
    uint32_t pad;
    uint64_t C;
    calc_pad(len, CHIP_FEC_K, &pad, &C);
    return (uint64_t)CHIP_FEC_M * C / 1024;
}

// fn(t) for t < nt on the caller and nt - 1 fresh threads.  (A persistent
// team parked on a condition variable measured 30 % slower on the GPU box:
// woken workers pile onto the waker's cores, r9p_session.)
void run_threads(uint32_t nt, const std::function<void(uint32_t)> &fn) {
    std::vector<std::thread> pool;
    for (uint32_t t = 1; t < nt; ++t) pool.emplace_back(fn, t);
    fn(0);
    for (auto &th : pool) th.join();
}

// CHIP_ECIES_PREP=0: each object's scalar multiplications inside its host stage
bool ecies_prep_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_ECIES_PREP");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

// The ECIES key material of a slice's objects (host::ecies_prepare: two
// scalar multiplications each, no data) computed on nt threads while the
// caller waits for the slice's slot: the slot wait is host time the data
// stages cannot use, the key material is the part of them that does not
// need the data.  The caller claims objects too once its wait is over.
struct KeyPrep {
    std::vector<host::EciesKey> keys;
    std::vector<int> sts;
    std::atomic<uint64_t> next{0};
    uint64_t cnt = 0;
    const uint8_t *peer = nullptr, *eph = nullptr;  // eph: injected secrets of the slice's objects
    std::vector<std::thread> pool;
    void claim() {
        for (uint64_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < cnt;)
            sts[j] = host::ecies_prepare(peer, eph ? eph + 32 * j : nullptr, &keys[j]);
    }
    void start(uint32_t nt, const uint8_t *peer_, const uint8_t *eph_, uint64_t cnt_) {
        if (keys.size() < cnt_) keys.resize(cnt_), sts.resize(cnt_);
        peer = peer_, eph = eph_, cnt = cnt_;
        next.store(0, std::memory_order_relaxed);
        for (uint32_t t = 0; t < nt; ++t) pool.emplace_back([this] { claim(); });
    }
    void finish() {
        claim();
        for (auto &th : pool) th.join();
        pool.clear();
    }
    void wipe() {
        for (uint64_t j = 0; j < cnt; ++j) host::ecies_key_wipe(&keys[j]);
    }
    ~KeyPrep() {
        for (auto &th : pool) th.join();
        wipe();
    }
};

// CHIP_E2E_TRACE=1: where a chip_encode_host_batch call's wall time went
// (host work of the slices on their threads, waits for a slot's stream, the final
// drain), one line on stderr per call
struct CallTrace {
    bool on = [] {
        const char *v = std::getenv("CHIP_E2E_TRACE");
        return v && v[0] == '1';
    }();
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    double host = 0, host_max = 0, wait = 0, drain = 0, prep = 0;
    double now() const {
        return on ? std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() : 0.0;
    }
    void report(uint64_t slices, uint64_t S) const {
        if (!on) return;
        std::fprintf(stderr,
                     "[chip e2e] %llu slices of %llu: wall %.1f ms, host %.1f ms (slice max %.2f), "
                     "slot waits %.1f ms (with ECIES key prep %.1f ms), drain %.1f ms\n",
                     (unsigned long long)slices, (unsigned long long)S, now() * 1e3, host * 1e3, host_max * 1e3,
                     wait * 1e3, prep * 1e3, drain * 1e3);
    }
};

// a slice waiting for its nodes: cnt objects, compact buffers at hnodes + j * nstride
struct SplitPending {
    const SplitGeo *g = nullptr;
    uint8_t *out = nullptr;
    uint64_t pitch = 0, cnt = 0, nstride = 0;
    const uint8_t *hnodes = nullptr;
    void scatter(uint64_t j) const {
        const uint8_t *src = hnodes + j * nstride;
        uint8_t *dst = out + j * pitch;
        for (const SplitGeo::Run &r : g->runs) std::memcpy(dst + r.dst, src + r.src, r.len);
    }
};

// Device part of one slice of chip_encode_host_batch: cnt objects of cur_n
// bytes at src (host, pitch src_pitch) -> zfec -> bao -> out (host).  With
// split (Zfec|Bao only), the data region of every stream is the host's
// (SplitGeo): the region's nodes go to sl.hnodes, the tail to out.
int batch_slice_device(Slot &sl, uint8_t format, const GfPlan *plan, const chip_encode_info &inf,
                       const uint8_t *src, uint64_t src_pitch, uint64_t cur_n, uint64_t zlen, uint64_t final_len,
                       uint64_t cnt, uint8_t *out, uint64_t out_pitch, uint8_t *hashes, uint64_t stream_off,
                       const SplitGeo *split = nullptr, bool from_rows = false) {
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    // the streams 56 B into their rows: every chunk and node on a 64-B boundary
    // (K13, and K3 / the content mode for Bao alone; not KS, below 513 chunks)
    const bool any8 = bao && zlen &&
                      (zfec ? zfec_bao_any8(inf.chunk_len, cnt) : (zlen + 1023) / 1024 > KS_MAX_N);
    const uint64_t soff = any8 ? stream_off : 0;
    const uint64_t n_al = row_pitch(cur_n), z_al = row_pitch(zlen), f_al = row_pitch(final_len + soff);
    uint8_t *d_in = static_cast<uint8_t *>(sl.in.p);
    if (from_rows && split && cur_n) {
        // the host stage wrote each object's zfec input into its stream's chunk slots
        // in out: the data regions come over and the chunks are gathered into rows
        const uint64_t t_al = row_pitch(split->t0);
        uint8_t *d_sin = static_cast<uint8_t *>(sl.sin.p);
        CHIP_HIP(hipMemcpy2DAsync(d_sin, t_al, out, out_pitch, split->t0, cnt, hipMemcpyHostToDevice, sl.stream));
        CHIP_HIP(bao_gather_rows(d_sin, t_al, split->N, cnt, cur_n, d_in, n_al, sl.stream));
    } else if (cur_n) {
        CHIP_HIP(hipMemcpy2DAsync(d_in, n_al, src, src_pitch, cur_n, cnt, hipMemcpyHostToDevice, sl.stream));
    }
    const uint8_t *d_cur = d_in;
    uint64_t cur_stride = n_al;
    if (zfec && bao && zlen) {  // fused: shards written into the bao streams, hashed in place
        uint8_t *d_str = static_cast<uint8_t *>(sl.out.p) + soff;
        CHIP_HIP(zfec_bao_dev(d_in, n_al, cur_n, cnt, inf.chunk_len, d_str, f_al, static_cast<uint8_t *>(sl.hash.p),
                              sl.scratch.p, sl.stream));
        CHIP_HIP(hipMemcpyAsync(hashes, sl.hash.p, 32 * cnt, hipMemcpyDeviceToHost, sl.stream));
        if (split) {
            const uint64_t ns = 64 * split->nb;
            if (ns) {
                CHIP_HIP(bao_data_nodes(d_str, f_al, split->N, split->nd, cnt, static_cast<uint8_t *>(sl.nodes.p), ns,
                                        sl.stream));
                CHIP_HIP(hipMemcpyAsync(sl.hnodes.p, sl.nodes.p, cnt * ns, hipMemcpyDeviceToHost, sl.stream));
            }
            CHIP_HIP(hipMemcpy2DAsync(out + split->t0, out_pitch, d_str + split->t0, f_al, final_len - split->t0, cnt,
                                      hipMemcpyDeviceToHost, sl.stream));
        } else if (final_len) {
            CHIP_HIP(hipMemcpy2DAsync(out, out_pitch, d_str, f_al, final_len, cnt, hipMemcpyDeviceToHost, sl.stream));
        }
        return CHIP_OK;
    }
    if (zfec) {
        GfLaunch L{d_in, static_cast<uint8_t *>(sl.mid.p), n_al, z_al, cur_n, inf.chunk_len, cnt};
        CHIP_HIP(gf_apply(*plan, L, sl.stream));
        d_cur = static_cast<const uint8_t *>(sl.mid.p);
        cur_stride = z_al;
    }
    const uint8_t *d_res = d_cur;
    uint64_t res_stride = cur_stride;
    if (bao) {
        CHIP_HIP(bao_encode_dev(d_cur, cur_stride, zlen, cnt, static_cast<uint8_t *>(sl.out.p) + soff, f_al,
                                static_cast<uint8_t *>(sl.hash.p), sl.scratch.p, sl.stream));
        d_res = static_cast<const uint8_t *>(sl.out.p) + soff;
        res_stride = f_al;
        CHIP_HIP(hipMemcpyAsync(hashes, sl.hash.p, 32 * cnt, hipMemcpyDeviceToHost, sl.stream));
    } else {
        for (uint64_t o = 0; o < cnt; ++o) std::memset(hashes + 32 * o, 0, 32);
    }
    if (final_len)
        CHIP_HIP(hipMemcpy2DAsync(out, out_pitch, d_res, res_stride, final_len, cnt, hipMemcpyDeviceToHost,
                                  sl.stream));
    return CHIP_OK;
}

}  // namespace

int chip_encode_host_batch(uint8_t format, const uint8_t *pubkey, uint64_t pubkey_len,
                           const chip_ecies_inject *inject, const uint8_t *in, uint64_t n, uint64_t count,
                           uint64_t in_stride, uint8_t *out, uint64_t out_stride, uint64_t *out_len,
                           uint8_t *hashes, chip_encode_info *info, uint32_t nslots, uint64_t slice_bytes,
                           uint32_t host_threads) {
    if ((!in && n && count) || (!out_len && count) || (!hashes && count)) return CHIP_ERR_INVALID_ARG;
    if ((format & CHIP_FORMAT_ECIES) && !pubkey) return CHIP_ERR_INVALID_ARG;
    if (count > 1 && in_stride < n) return CHIP_ERR_INVALID_ARG;
    if (count == 0) return CHIP_OK;
    const bool hs = has_host_stages(format);
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    // sizes: exact without host stages, bounds with them
    const uint64_t h_max = hs ? host_stage_max(format, n) : n;
    chip_encode_info inf_max;
    uint64_t zlen_max, final_max;
    int st = encode_info_for(format, n, h_max, 0, 0, &inf_max, &zlen_max, &final_max);
    if (st != CHIP_OK && !hs) return st;
    if (hs) {  // bound without the slice-count check (a smaller object may still pass it)
        uint32_t pad;
        uint64_t C;
        calc_pad(h_max, CHIP_FEC_K, &pad, &C);
        zlen_max = zfec ? (uint64_t)CHIP_FEC_M * C : h_max;
        final_max = bao ? bao_encoded_len(zlen_max) : zlen_max;
    }
    if (count > 1 && out_stride < final_max) return CHIP_ERR_BUFFER_TOO_SMALL;
    if (final_max && !out) return CHIP_ERR_BUFFER_TOO_SMALL;

    if (!hs && !zfec && !bao) {  // format 0: identity, nothing for the device to do
        for (uint64_t o = 0; o < count; ++o) {
            if (n) std::memcpy(out + o * out_stride, in + o * in_stride, n);
            std::memset(hashes + 32 * o, 0, 32);
            out_len[o] = n;
            if (info) info[o] = inf_max;
        }
        return CHIP_OK;
    }
    Ctx *c = nullptr;
    if (zfec || bao) {
        st = ctx_get(&c);
        if (st != CHIP_OK) return st;
    }
    nslots = nslots < 1 ? 3 : (nslots > 8 ? 8 : nslots);
    if (slice_bytes == 0) slice_bytes = 256ull << 20;
    uint32_t T = host_threads ? host_threads : std::max(1u, std::thread::hardware_concurrency());
    T = std::min<uint32_t>(T, 64);
    const uint64_t h_al = (h_max + 15) / 16 * 16;  // pinned staging pitch
    uint64_t S = slice_bytes / (h_max ? h_max : 1);
    S = S < 1 ? 1 : S;
    // host work per object (host stages, split copy-back): a slice of at least half as
    // many objects as host threads is rounded up to a multiple of them (equal shares)
    if ((hs || (zfec && bao)) && S >= (T + 1) / 2) S = (S + T - 1) / T * T;
    S = S > count ? count : S;
    // split copy-back (SplitGeo): Zfec|Bao streams of at least 2 chunks
    const bool split_fmt = zfec && bao && c && e2e_split_on() && zlen_max >= 2048;
    // ...and with ECIES, the host stage writes each stream's data region straight
    // into out (pinned), which the device then reads: no staging copy at all
    const bool direct_fmt = split_fmt && hs && stream_encrypt_on() && direct_rows_on() && out && host_pinned(out);
    SplitGeos geos;
    const uint64_t soff_cfg = stream_offset();  // where K13's streams sit in the slot rows (this call)
    if (c) {
        if (c->slots.size() < nslots) c->slots.resize(nslots);
        for (uint32_t k = 0; k < nslots; ++k) {
            Slot &sl = c->slots[k];
            if (!sl.stream) CHIP_HIP(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
            CHIP_HIP(grow(sl.in, S * row_pitch(h_max)));
            if (zfec && !bao) CHIP_HIP(grow(sl.mid, S * row_pitch(zlen_max)));  // Zfec|Bao: fused
            if (bao) {
                CHIP_HIP(grow(sl.out, S * row_pitch(final_max + soff_cfg)));
                CHIP_HIP(grow(sl.scratch, zfec ? std::max(zfec_bao_scratch_len(zlen_max, S), bao_scratch_len(zlen_max, S))
                                                : bao_scratch_len(zlen_max, S)));
            }
            CHIP_HIP(grow(sl.hash, S * 32));
            if (hs) CHIP_HIP(grow_pinned(sl.stage, S * h_al));
            if (split_fmt) {  // the data region's nodes: fewer than the stream's N chunks
                CHIP_HIP(grow(sl.nodes, S * 64 * (zlen_max / 1024)));
                CHIP_HIP(grow_pinned(sl.hnodes, S * 64 * (zlen_max / 1024)));
                if (direct_fmt) CHIP_HIP(grow(sl.sin, S * row_pitch(geos.get(zlen_max / 1024).t0)));
            }
        }
    }
    const std::vector<uint8_t> enc = zfec_enc_matrix(CHIP_FEC_K, CHIP_FEC_M);
    std::vector<SplitPending> pend(nslots);  // per slot: the slice whose nodes are still to be placed
    std::vector<uint8_t> stage_host;  // host stages without a device part
    if (!c) stage_host.resize(S * h_al);
    std::vector<uint64_t> len(S), bc(S), be(S);
    std::vector<int> sts(S);
    std::vector<uint8_t> in_rows(S);  // object's data region written straight into out (direct)
    CallTrace tr;
    std::vector<Scratch> scratch(T);  // per host thread, reused across slices
    // ECIES on the streaming path: the receiver key parsed once, each slice's
    // key material prepared during its slot wait (KeyPrep)
    const bool prep = (format & CHIP_FORMAT_ECIES) && stream_encrypt_on() && ecies_prep_on();
    uint8_t peer[65];
    if (prep) {
        st = host::ecies_peer(pubkey, pubkey_len, peer);
        if (st != CHIP_OK) return st;
    }
    KeyPrep kp;
    auto drain = [&]() {
        if (c)
            for (uint32_t k = 0; k < nslots; ++k) (void)hipStreamSynchronize(c->slots[k].stream);
    };
    const uint64_t nslices = (count + S - 1) / S;
    for (uint64_t i = 0; i < nslices; ++i) {
        Slot *sl = c ? &c->slots[i % nslots] : nullptr;
        const uint64_t o0 = i * S, cnt = (count - o0) < S ? (count - o0) : S;
        if (prep)
            kp.start(std::min<uint64_t>(T, cnt), peer,
                     inject && inject->ephemeral_sk ? inject->ephemeral_sk + 32 * o0 : nullptr, cnt);
        const double t_a = tr.now();
        if (sl && i >= nslots) {
            const hipError_t e = hipStreamSynchronize(sl->stream);  // slot's previous slice is done
            if (e != hipSuccess) {
                kp.finish();
                set_device_error(e);
                return CHIP_ERR_DEVICE;
            }
        }
        tr.wait += tr.now() - t_a;
        if (prep) {
            kp.finish();
            tr.prep += tr.now() - t_a;
            for (uint64_t j = 0; j < cnt; ++j)
                if (kp.sts[j] != CHIP_OK) {
                    drain();
                    return kp.sts[j];
                }
        }
        const uint8_t *src = in + o0 * in_stride;
        uint64_t src_pitch = count > 1 ? in_stride : n;
        uint64_t cur_n = n;
        bool uniform = true, rows = false;
        SplitPending &pp = pend[i % nslots];  // this slot's previous slice (its stream is done)
        if (hs || split_fmt) {
            // on T threads while earlier slices run on the device: the nodes of this
            // slot's previous slice into place, then this slice's host stages and the
            // data region of its streams (split copy-back)
            uint8_t *stage = hs ? (sl ? static_cast<uint8_t *>(sl->stage.p) : stage_host.data()) : nullptr;
            const uint32_t nt = (uint32_t)std::min<uint64_t>(T, std::max(cnt, pp.g ? pp.cnt : 0));
            // the geometry an incompressible object's stream will have: ECIES places
            // its chunks block by block against it (host::ChunkSink)
            const uint64_t n_pred = split_fmt && hs ? split_chunks(h_max) : 0;
            const SplitGeo *g_pred = n_pred >= 2 ? &geos.get(n_pred) : nullptr;
            const bool direct = direct_fmt && g_pred;
            auto work = [&](uint32_t t) {
                Scratch &tmp = scratch[t];
                if (pp.g)
                    for (uint64_t j = t; j < pp.cnt; j += nt) pp.scatter(j);
                for (uint64_t j = t; j < cnt; j += nt) {
                    const uint64_t o = o0 + j;
                    const uint8_t *obj = in + o * in_stride;
                    uint64_t olen = n, filled = 0;
                    uint8_t *row = out + o * out_stride;
                    in_rows[j] = 0;
                    if (hs) {
                        const host::ChunkSink sink{row, g_pred ? g_pred->coff.data() : nullptr,
                                                   g_pred ? g_pred->nd : 0, direct, 1024 * n_pred};
                        sts[j] = host_stages_into(format, pubkey, pubkey_len,
                                                  inject && inject->ephemeral_sk ? inject->ephemeral_sk + 32 * o
                                                                                 : nullptr,
                                                  inject && inject->nonce ? inject->nonce + 16 * o : nullptr, obj, n,
                                                  direct ? nullptr : stage + j * h_al, h_al, tmp, &len[j], &bc[j],
                                                  &be[j], g_pred ? &sink : nullptr, &filled,
                                                  prep ? &kp.keys[j] : nullptr);
                        if (sts[j] != CHIP_OK) continue;
                        olen = len[j];
                        if (direct) {
                            if (split_chunks(olen) == n_pred) {  // the data region is complete in out
                                host::fill_chunk_range(row, g_pred->coff.data(), filled, g_pred->nd, nullptr, 0);
                                in_rows[j] = 1;
                                continue;
                            }
                            // another geometry (compressible input): the output back from the slots
                            host::gather_chunks(stage + j * h_al, row, g_pred->coff.data(), olen);
                            filled = 0;
                        }
                        obj = stage + j * h_al;
                    }
                    // the stream's header and data chunks (a ragged slice copies its
                    // streams back whole over this; chunks placed against a wrong
                    // prediction lie inside the stream and are overwritten too)
                    if (split_fmt) {
                        const uint64_t N = split_chunks(olen);
                        if (N >= 2) {
                            const SplitGeo &g = geos.get(N);
                            if (filled > 1 && N == n_pred) {  // chunks [1, filled) are in place
                                host::fill_data_chunks(row, g.coff.data(), 1, 1024 * N, obj, olen);
                                host::fill_chunk_range(row, g.coff.data(), filled, g.nd, obj, olen);
                            } else {
                                host::fill_data_chunks(row, g.coff.data(), g.nd, 1024 * N, obj, olen);
                            }
                        }
                    }
                }
            };
            const double t_h = tr.now();
            run_threads(nt, work);
            const double dh = tr.now() - t_h;
            tr.host += dh;
            tr.host_max = std::max(tr.host_max, dh);
            pp = SplitPending{};
            if (prep) kp.wipe();
            if (hs) {
                for (uint64_t j = 0; j < cnt; ++j)
                    if (sts[j] != CHIP_OK) {
                        drain();
                        return sts[j];
                    }
                src = stage;
                src_pitch = h_al;
                cur_n = len[0];
                for (uint64_t j = 1; j < cnt; ++j) uniform &= len[j] == cur_n;
                rows = direct && uniform;
                for (uint64_t j = 0; j < cnt; ++j) rows &= in_rows[j] != 0;
                if (direct && !rows)  // a ragged slice: from the staging rows, as without `direct`
                    for (uint64_t j = 0; j < cnt; ++j)
                        if (in_rows[j])
                            host::gather_chunks(stage + j * h_al, out + (o0 + j) * out_stride,
                                                g_pred->coff.data(), len[j]);
            }
        }
        if (!hs) {
            for (uint64_t j = 0; j < cnt; ++j) len[j] = n, bc[j] = be[j] = 0;
        }
        // per-object EncodeInfo (identical for a uniform slice)
        for (uint64_t j = 0; j < cnt; ++j) {
            chip_encode_info inf;
            uint64_t zl, fl;
            st = encode_info_for(format, n, len[j], bc[j], be[j], &inf, &zl, &fl);
            if (st != CHIP_OK) {
                drain();
                return st;
            }
            out_len[o0 + j] = fl;
            if (info) info[o0 + j] = inf;
        }
        if (!sl) {  // host stages only (no Zfec/Bao bit)
            for (uint64_t j = 0; j < cnt; ++j) {
                std::memcpy(out + (o0 + j) * out_stride, src + j * src_pitch, len[j]);
                std::memset(hashes + 32 * (o0 + j), 0, 32);
            }
            continue;
        }
        if (uniform) {
            chip_encode_info inf;
            uint64_t zl, fl;
            (void)encode_info_for(format, n, cur_n, 0, 0, &inf, &zl, &fl);
            const GfPlan p2 = encode_plan(CHIP_FEC_K, CHIP_FEC_M, inf.chunk_len, enc);
            const SplitGeo *g = split_fmt && zl >= 2048 ? &geos.get(zl / 1024) : nullptr;
            const uint64_t opitch = count > 1 ? out_stride : fl;
            st = batch_slice_device(*sl, format, &p2, inf, src, src_pitch, cur_n, zl, fl, cnt, out + o0 * out_stride,
                                    opitch, hashes + 32 * o0, soff_cfg, g, rows);
            if (st != CHIP_OK) {
                drain();
                return st;
            }
            if (g)
                pp = SplitPending{g, out + o0 * out_stride, opitch, cnt, 64 * g->nb,
                                  static_cast<const uint8_t *>(sl->hnodes.p)};
        } else {  // ragged host-stage output (compressible data): one object at a time
            for (uint64_t j = 0; j < cnt; ++j) {
                chip_encode_info inf;
                uint64_t zl, fl;
                (void)encode_info_for(format, n, len[j], 0, 0, &inf, &zl, &fl);
                const GfPlan pj = encode_plan(CHIP_FEC_K, CHIP_FEC_M, inf.chunk_len, enc);
                st = batch_slice_device(*sl, format, &pj, inf, src + j * src_pitch, src_pitch, len[j], zl, fl, 1,
                                        out + (o0 + j) * out_stride, fl, hashes + 32 * (o0 + j), soff_cfg);
                if (st != CHIP_OK) {
                    drain();
                    return st;
                }
            }
        }
    }
    const double t_d = tr.now();
    if (c)
        for (uint32_t k = 0; k < nslots; ++k) CHIP_HIP(hipStreamSynchronize(c->slots[k].stream));
    tr.drain = tr.now() - t_d;
    tr.report(nslices, S);
    // the nodes of the last slices into place
    for (uint32_t k = 0; k < nslots; ++k) {
        if (!pend[k].g) continue;
        const uint32_t nt = (uint32_t)std::min<uint64_t>(T, pend[k].cnt);
        run_threads(nt, [&pend, k, nt](uint32_t t) {
            for (uint64_t j = t; j < pend[k].cnt; j += nt) pend[k].scatter(j);
        });
    }
    return CHIP_OK;
}

}  // extern "C"
