// api_single.cpp — one object from host memory, for latency: encode() at
// Zfec|Bao or Bao and decode() of a bao stream on KM (multi_kernels.hip; KS,
// small_kernels.hip, up to 64 chunks), and one object's zfec alone
// (parity_kernel<1> / the K1 decode on pinned memory).
//
// A single object's call was the kernel's own 65-115 us (K13: 32 waves for
// a 1 MiB object) and PCIe for every stream byte both ways (profiles/
// r10zm_session, r11a).  Here the device runs KM (a quad of lanes per
// compression, all CUs), and the copies move only what the host cannot make:
//
//  * zero-copy: the host copies the input (or the stream to verify) into
//    pinned memory on the GPU's NUMA node on a few threads, and the kernels
//    read it over PCIe themselves and write their outputs there.  No DMA and
//    no copy-engine handoff sits on the critical path (each cost ~10-14 us
//    besides the transfer, profiles/r11c_session), and the transfer overlaps
//    the hashing.
//  * encode: the host writes the stream's header and the chunks it already
//    holds (the content, or the data shards = the zero-padded input) into the
//    caller's buffer while the device hashes; only the parity region [t0,
//    end) and the parent nodes in front of t0 (KM writes those compactly)
//    come back.  At level 12 that is 1.13 of the stream's 2.2 MB per 1 MiB;
//    for bao of the content only the nodes (1/16 of the content).
//  * decode: every stream byte goes up (all of it is hashed), and the content
//    the caller gets is gathered from the caller's own input by the host while
//    the device verifies; only the verdict comes back, and the gathered bytes
//    are wiped if it is a mismatch.
#include "api_common.hpp"

#include <chrono>
#include <map>
#include <mutex>

namespace chip {
namespace api {

namespace {

// The host-made part of a stream of N chunks whose first `nh` chunks the host
// holds: their slots, the parent-node runs between them (dst: stream offset,
// src: offset in KM's compact node buffer) and the end t0 of that region.
struct HostGeo {
    uint64_t N = 0, nh = 0, zl = 0, t0 = 8, nbytes = 0;  // nbytes: compact node bytes
    std::vector<uint64_t> coff;  // slots of chunks [0, nh), then (tail) of chunks [nh, N)
    struct Run {
        uint64_t dst, src, len;
    };
    std::vector<Run> runs;   // the nodes in front of t0: stream offset, compact offset, bytes
    std::vector<Run> truns;  // the nodes past t0 (tail only): stream offset, -, bytes
};

const HostGeo &host_geo(uint64_t zl, uint64_t nh) {
    thread_local std::map<std::pair<uint64_t, uint64_t>, HostGeo> cache;
    auto key = std::make_pair(zl, nh);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (cache.size() >= 8) cache.clear();
    HostGeo g;
    g.zl = zl;
    g.N = n_chunks_of(zl);
    g.nh = nh;
    g.coff.resize(nh);
    uint64_t prev_end = 8, src = 0;
    for (uint64_t i = 0; i < nh; ++i) {
        g.coff[i] = bao_chunk_offset(i, g.N);
        if (g.coff[i] > prev_end) {
            g.runs.push_back({prev_end, src, g.coff[i] - prev_end});
            src += g.coff[i] - prev_end;
        }
        prev_end = g.coff[i] + std::min<uint64_t>(1024, zl - 1024 * i);
    }
    g.t0 = prev_end;
    g.nbytes = src;
    if (nh < g.N) {  // the tail: chunk slots and the node runs between them
        g.coff.resize(g.N);
        for (uint64_t i = nh; i < g.N; ++i) {
            g.coff[i] = bao_chunk_offset(i, g.N);
            if (g.coff[i] > prev_end) g.truns.push_back({prev_end, 0, g.coff[i] - prev_end});
            prev_end = g.coff[i] + std::min<uint64_t>(1024, zl - 1024 * i);
        }
    }
    return cache.emplace(key, std::move(g)).first->second;
}

// host copy threads for `bytes`: one per 128 KiB, at most CHIP_ZC_THREADS
// (default 8; an A/B knob: one thread streams ~80 GB/s into pinned memory from
// a cached source, tools/bar_probe)
int copy_parts(uint64_t bytes) {
    static const uint64_t cap = [] {
        const char *v = std::getenv("CHIP_ZC_THREADS");
        const int t = v ? std::atoi(v) : 8;
        return (uint64_t)(t >= 1 && t <= 32 ? t : 8);
    }();
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(cap, bytes >> 17));
}
int host_parts(uint64_t nc) { return copy_parts(nc * 1024); }


// a pinned host allocation as the device addresses it (looked up once per
// allocation: the runtime call takes its allocation lock)
template <class T>
T *dev_ptr(void *host) {
    thread_local void *last_host[2] = {nullptr, nullptr}, *last_dev[2] = {nullptr, nullptr};
    for (int i = 0; i < 2; ++i)
        if (last_host[i] == host) return static_cast<T *>(last_dev[i]);
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        (void)hipGetLastError();
        d = host;  // UVA: the same address
    }
    last_host[1] = last_host[0];
    last_dev[1] = last_dev[0];
    last_host[0] = host;
    last_dev[0] = d;
    return static_cast<T *>(d);
}

// n bytes into pinned memory on a few threads (streaming stores: only the
// device reads them next)
void copy_in(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const int parts = copy_parts(n);
    host::par_for(parts, [&](int i) {
        const uint64_t a = (n * i / parts) & ~uint64_t(63), b = i + 1 == parts ? n : (n * (i + 1) / parts) & ~uint64_t(63);
        host::ring_copy(dst + a, src + a, b - a);
    });
}

void copy_out(uint8_t *dst, const uint8_t *src, uint64_t n) {
    const int parts = copy_parts(n);
    host::par_for(parts, [&](int i) {
        const uint64_t a = n * i / parts, b = n * (i + 1) / parts;
        std::memcpy(dst + a, src + a, b - a);
    });
}


// a decode's `meanwhile` (the ECIES key) as a task beside the content gather
// rather than after it: CHIP_DEC_SIDE=0 turns it off (an A/B knob)
bool dec_side_task() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_DEC_SIDE");
        return !(e && e[0] == '0');
    }();
    return on;
}

// the largest stream (chunks) a single call runs on KS rather than KM:
// CHIP_KS_SINGLE_MAX (64 .. 512, an A/B knob), default 64
uint64_t ks_single_max() {
    static const uint64_t v = [] {
        const char *e = std::getenv("CHIP_KS_SINGLE_MAX");
        const long x = e ? std::atol(e) : 64;
        return (uint64_t)(x >= 64 && x <= (long)KS_MAX_N ? x : 64);
    }();
    return v;
}

// KS (small_kernels.hip, one workgroup) for a stream of at most 64 chunks,
// zero-copy too: the input from pinned memory, the whole stream and the hash
// written there by the kernel (at most ~70 KB), copied out after.
int single_encode_ks(Ctx *c, const uint8_t *cur, uint64_t cur_n, uint64_t C, uint64_t final_len, uint8_t *out,
                     uint8_t hash[32]) {
    Trace trace("encode ks");
    const uint64_t hash_at = (final_len + 63) & ~uint64_t(63);
    CHIP_HIP(grow_pinned_local(c->hin, cur_n + 16));  // the kernel's 16-B source loads stay inside
    CHIP_HIP(grow_pinned_local(c->hout, hash_at + 64));
    uint8_t *hin = static_cast<uint8_t *>(c->hin.p), *hout = static_cast<uint8_t *>(c->hout.p);
    if (cur != hin) std::memcpy(hin, cur, cur_n);
    const uint8_t *d_in = dev_ptr<const uint8_t>(hin);
    uint8_t *d_out = dev_ptr<uint8_t>(hout);
    if (C) CHIP_HIP(small_zfec_bao_dev(d_in, 0, cur_n, 1, C, d_out, 0, d_out + hash_at, c->stream));
    else CHIP_HIP(small_bao_encode_dev(d_in, 0, cur_n, 1, d_out, 0, d_out + hash_at, c->stream));
    trace.mark("launch");
    CHIP_HIP(hipStreamSynchronize(c->stream));
    trace.mark("sync");
    std::memcpy(out, hout, final_len);
    std::memcpy(hash, hout + hash_at, 32);
    trace.mark("copy out");
    return CHIP_OK;
}

}  // namespace

int single_encode_km(Ctx *c, const uint8_t *cur, uint64_t cur_n, uint64_t C, uint64_t final_len, uint8_t *out,
                     uint8_t hash[32]) {
    if (n_chunks_of(C ? (uint64_t)CHIP_FEC_M * C : cur_n) <= ks_single_max())
        return single_encode_ks(c, cur, cur_n, C, final_len, out, hash);
    Trace trace("encode");
    const bool zfec = C > 0;
    const uint64_t zl = zfec ? (uint64_t)CHIP_FEC_M * C : cur_n;
    const uint64_t N = n_chunks_of(zl), nh = zfec ? N / 2 : N;
    const HostGeo &g = host_geo(zl, nh);
    // pinned outputs: [the stream image from t0][the compact nodes][the hash]
    const uint64_t tail_len = final_len - g.t0, nodes_at = (tail_len + 63) & ~uint64_t(63);
    const uint64_t hash_at = (nodes_at + g.nbytes + 63) & ~uint64_t(63);
    CHIP_HIP(grow_pinned_local(c->hin, cur_n + 16));  // the kernels' 16-B source loads stay inside
    CHIP_HIP(grow_pinned_local(c->hout, hash_at + 64));
    if (zfec) CHIP_HIP(grow(c->out, final_len));
    CHIP_HIP(grow(c->scratch, km_scratch_len(zl)));
    trace.mark("buffers");
    uint8_t *hin = static_cast<uint8_t *>(c->hin.p), *hout = static_cast<uint8_t *>(c->hout.p);
    if (cur != hin) copy_in(hin, cur, cur_n);  // (the host stages may have written it there already)
    trace.mark("copy in");
    const uint8_t *d_in = dev_ptr<const uint8_t>(hin);
    uint8_t *d_out = dev_ptr<uint8_t>(hout);
    if (zfec) {
        if (!c->ev_km) CHIP_HIP(hipEventCreateWithFlags(&c->ev_km, hipEventDisableTiming));
        CHIP_HIP(km_zfec_bao_dev(d_in, cur_n, C, static_cast<uint8_t *>(c->out.p), d_out + nodes_at, d_out, g.t0,
                                 d_out + hash_at, c->scratch.p, c->stream, c->ev_km));
    } else
        CHIP_HIP(km_bao_encode_dev(d_in, cur_n, d_out + nodes_at, d_out + hash_at, c->scratch.p, c->stream));
    trace.mark("launch");
    // meanwhile: the header and the chunks the host holds, on a few threads
    advise_huge(out, final_len);
    for (int b = 0; b < 8; ++b) out[b] = static_cast<uint8_t>(zl >> (8 * b));
    const int parts = host_parts(nh);
    host::par_for(parts, [&](int i) {
        const uint64_t a = nh * i / parts, b = nh * (i + 1) / parts;
        if (zfec) host::fill_chunk_range(out, g.coff.data(), a, b, cur, cur_n);
        else host::gather_chunks_to_slots(out, g.coff.data() + a, cur + 1024 * a, std::min(cur_n, 1024 * b) - 1024 * a);
    });
    trace.mark("host chunks");
    if (zfec) {  // the parity chunks are final once the parity kernel is done: out while KM hashes
        CHIP_HIP(hipEventSynchronize(c->ev_km));
        trace.mark("parity done");
        const int pp = host_parts(N - nh);
        host::par_for(pp, [&](int i) {
            const uint64_t a = nh + (N - nh) * i / pp, b = nh + (N - nh) * (i + 1) / pp;
            for (uint64_t k = a; k < b; ++k) std::memcpy(out + g.coff[k], hout + (g.coff[k] - g.t0), 1024);
        });
        trace.mark("parity out");
    }
    CHIP_HIP(hipStreamSynchronize(c->stream));
    trace.mark("sync");
    if (!zfec && tail_len) copy_out(out + g.t0, hout, tail_len);
    // the node runs (thousands of 64-B pieces per MiB) on a few threads
    const uint64_t nr = g.runs.size(), nt = zfec ? g.truns.size() : 0;
    const int rp = (int)std::max<uint64_t>(1, std::min<uint64_t>(8, (nr + nt) / 256));
    host::par_for(rp, [&](int i) {
        for (uint64_t k = nr * i / rp; k < nr * (i + 1) / rp; ++k) {
            const HostGeo::Run &r = g.runs[k];
            std::memcpy(out + r.dst, hout + nodes_at + r.src, r.len);
        }
        for (uint64_t k = nt * i / rp; k < nt * (i + 1) / rp; ++k) {
            const HostGeo::Run &r = g.truns[k];
            std::memcpy(out + r.dst, hout + (r.dst - g.t0), r.len);
        }
    });
    std::memcpy(hash, hout + hash_at, 32);
    trace.mark("copy out");
    return CHIP_OK;
}

int single_zfec_encode_zc(Ctx *c, const uint8_t *in, uint64_t n, uint64_t C, uint8_t *out) {
    Trace trace("zfec");
    CHIP_HIP(grow_pinned_local(c->hin, n + 16));
    CHIP_HIP(grow_pinned_local(c->hout, 4 * C));
    uint8_t *hin = static_cast<uint8_t *>(c->hin.p), *hout = static_cast<uint8_t *>(c->hout.p);
    if (in != hin) copy_in(hin, in, n);
    trace.mark("copy in");
    CHIP_HIP(zc_zfec_parity_dev(dev_ptr<const uint8_t>(hin), n, C, dev_ptr<uint8_t>(hout), c->stream));
    trace.mark("launch");
    // meanwhile: the data shards are the input, zero padded to 4 C
    advise_huge(out, 8 * C);
    copy_out(out, in, n);
    std::memset(out + n, 0, 4 * C - n);
    trace.mark("data shards");
    CHIP_HIP(hipStreamSynchronize(c->stream));
    trace.mark("sync");
    copy_out(out + 4 * C, hout, 4 * C);
    trace.mark("copy out");
    return CHIP_OK;
}

int single_zfec_decode_zc(Ctx *c, uint32_t k, uint32_t m, const uint8_t *const *shares,
                          const std::vector<uint32_t> &sel, uint64_t C, uint8_t *dst, uint64_t olen,
                          const std::function<void()> &meanwhile) {
    Trace trace("zfec decode");
    const uint64_t kc = (uint64_t)k * C;
    CHIP_HIP(grow_pinned_local(c->hin, kc));
    CHIP_HIP(grow_pinned_local(c->hout, kc));
    uint8_t *hin = static_cast<uint8_t *>(c->hin.p), *hout = static_cast<uint8_t *>(c->hout.p);
    // the k shares side by side at s * C, cut into equal runs across the copy threads
    const int parts = copy_parts(kc);
    host::par_for(parts, [&](int i) {
        uint64_t a = (kc * i / parts) & ~uint64_t(63);
        const uint64_t b = i + 1 == parts ? kc : (kc * (i + 1) / parts) & ~uint64_t(63);
        while (a < b) {
            const uint64_t s = a / C, o = a % C, len = std::min(b - a, C - o);
            host::ring_copy(hin + a, shares[s] + o, len);
            a += len;
        }
    });
    trace.mark("copy in");
    std::vector<uint64_t> slot_off(k);
    for (uint32_t s = 0; s < k; ++s) slot_off[s] = (uint64_t)s * C;
    int st = zfec_decode_device(k, m, dev_ptr<const uint8_t>(hin), 0, slot_off, sel, C, 1, dev_ptr<uint8_t>(hout),
                                0, c->stream);
    if (st != CHIP_OK) return st;
    trace.mark("launch");
    advise_huge(dst, olen);
    if (meanwhile) meanwhile();
    CHIP_HIP(hipStreamSynchronize(c->stream));
    trace.mark("sync");
    if (olen) copy_out(dst, hout, olen);  // (dst may be null for an empty result)
    trace.mark("copy out");
    return CHIP_OK;
}

int single_decode_km(Ctx *c, const uint8_t *in, uint64_t len, uint64_t n, const uint8_t *hash, uint8_t *dst,
                     uint64_t olen, const std::function<void()> &meanwhile, const std::function<void()> &gathered) {
    Trace trace("decode");
    const uint64_t blen = bao_encoded_len(n);
    if (blen > len) return CHIP_ERR_BAO_TRUNCATED;
    // pinned: [the expected hash][the status word][the stream at 64]
    CHIP_HIP(grow_pinned_local(c->hin, 64 + blen));
    CHIP_HIP(grow(c->scratch, km_scratch_len(n)));
    uint8_t *hin = static_cast<uint8_t *>(c->hin.p);
    trace.mark("buffers");
    std::memcpy(hin, hash, 32);
    volatile uint32_t *status = reinterpret_cast<volatile uint32_t *>(hin + 32);
    *status = 0;
    copy_in(hin + 64, in, blen);
    trace.mark("copy in");
    uint8_t *d = dev_ptr<uint8_t>(hin);
    if (n_chunks_of(n) <= ks_single_max())  // KS: one workgroup verifies the whole stream
        CHIP_HIP(small_bao_decode_dev(d + 64, 0, n, 1, d, nullptr, 0, 0, reinterpret_cast<uint32_t *>(d + 32),
                                      c->stream));
    else
        CHIP_HIP(km_bao_decode_dev(d + 64, n, d, nullptr, 0, reinterpret_cast<uint32_t *>(d + 32), c->scratch.p,
                                   c->stream));
    trace.mark("launch");
    // meanwhile: the content from the caller's own copy of the stream, and
    // `meanwhile` beside it as one more task of the same pool job
    advise_huge(dst, olen);
    const uint64_t nc = (olen + 1023) / 1024;
    const int parts = olen ? host_parts(nc) : 0;
    const bool side = meanwhile && parts > 1 && dec_side_task();
    if (parts) {
        const HostGeo &g = host_geo(n, nc);
        host::par_for(parts + side, [&](int i) {
            if (side && i == 0) return meanwhile();
            i -= side;
            const uint64_t a = nc * i / parts, b = nc * (i + 1) / parts;
            host::gather_chunks(dst + 1024 * a, in, g.coff.data() + a, std::min(olen, 1024 * b) - 1024 * a);
        });
    }
    trace.mark("host gather");
    if (meanwhile && !side) meanwhile();
    trace.mark("meanwhile");
    if (gathered) gathered();
    trace.mark("gathered");
    CHIP_HIP(hipStreamSynchronize(c->stream));
    trace.mark("sync");
    const uint32_t verdict = *status;
    if (verdict) {  // never hand back unverified content
        if (olen) std::memset(dst, 0, olen);
        return (int)verdict;
    }
    return CHIP_OK;
}

}  // namespace api
}  // namespace chip
