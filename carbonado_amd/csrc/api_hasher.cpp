// api_hasher.cpp — the streaming BaoHasher (utils.rs:104-137): appends into
// grow-in-place HBM, chunk CVs hashed during update(), the parents at
// finalize, freed hashers parked for reuse (bounded).  Shared declarations:
// api_common.hpp.
#include <mutex>

#include "api_common.hpp"

#include "hbm_alloc.hpp"

using namespace chip;
using namespace chip::api;

// Incremental (utils.rs:104-137 streams into bao's Encoder): update() appends
// to a grow-only HBM buffer and, asynchronously on the hasher's stream, hashes
// every chunk that bytes have arrived past (whole 64-chunk units, so each
// launch fills a wave per unit); finalize() hashes the last chunks, lays the
// content out in its slots and builds the parent levels from the chunk CVs.
struct chip_bao_hasher {
    std::mutex mu;
    hipStream_t stream = nullptr;   // copies (and finalize)
    hipStream_t hstream = nullptr;  // update()'s chunk hashing, behind the copies through `copied`
    hipEvent_t copied = nullptr;
    DevBuf content, enc, scratch, hash, cv0, cv1;
    // content and cv0 grow in place behind a reserved VA range (no copy, no
    // device sync per growth); va_* says which of them live there
    chip::hbm::Growable gcontent, gcv0;
    bool va_content = false, va_cv0 = false;
    uint64_t va_content_bytes = 0;  // first content VA reservation (1 GiB; CHIP_HASHER_VA_MIB at creation)
    int dev = -1;                   // device its streams and buffers live on
    uint64_t len = 0, enc_len = 0;
    uint64_t units = 0;  // 64-chunk units whose chunk CVs are in cv0
    bool finalized = false;
    uint8_t h[32] = {0};
};

namespace {

// 64-chunk units per update-time hashing launch (32 MiB); CHIP_HASHER_UNITS
// overrides it (0 = hash everything at finalize, as before round 3; A/B)
uint64_t hasher_batch_units() {
    static const uint64_t u = [] {
        const char *e = std::getenv("CHIP_HASHER_UNITS");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)512;
    }();
    return u;
}

// Freed hashers are kept, emptied, with their two streams, their event and
// their grown buffers, and handed to the next chip_bao_hasher_new on the same
// device: stream creation and destruction, a GiB of hipMalloc / hipFree and
// the in-place buffers' mappings cost milliseconds per hasher otherwise (a
// mapped VA range is reused as is, never remapped).  Bounded: at most
// HASHER_PARK_COUNT parked hashers, and their buffers together at most
// hasher_park_bytes() (CHIP_HASHER_PARK_MIB, 3 GiB by default: the 1 GiB
// content of the hasher bench, its 1.06 GiB stream and the CV buffers); a
// hasher that would take the pool past it is parked without its buffers
// (streams only), so hashing one large file does not keep its HBM for the
// rest of the process.  chip_bao_hasher_drop_cache frees them all.
// CHIP_HASHER_CACHE=0: off.
constexpr size_t HASHER_PARK_COUNT = 4;
std::mutex g_hasher_spare_mu;
std::vector<chip_bao_hasher *> g_hasher_spares;

uint64_t hasher_park_bytes() {
    static const uint64_t b = [] {
        const char *e = std::getenv("CHIP_HASHER_PARK_MIB");
        return (e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)3072) << 20;
    }();
    return b;
}

// device bytes a hasher holds (mapped VA pieces and plain buffers)
uint64_t hasher_bytes(const chip_bao_hasher *h) {
    uint64_t s = (h->va_content ? h->gcontent.mapped : h->content.cap) + (h->va_cv0 ? h->gcv0.mapped : h->cv0.cap);
    for (const DevBuf *b : {&h->enc, &h->scratch, &h->hash, &h->cv1}) s += b->cap;
    return s;
}

// Free every buffer of a hasher whose work is done (its VA ranges retire).
void hasher_release_buffers(chip_bao_hasher *h) {
    if (h->va_content) h->gcontent.release();
    else if (h->content.p) (void)hipFree(h->content.p);
    if (h->va_cv0) h->gcv0.release();
    else if (h->cv0.p) (void)hipFree(h->cv0.p);
    for (DevBuf *b : {&h->enc, &h->scratch, &h->hash, &h->cv1})
        if (b->p) (void)hipFree(b->p);
    for (DevBuf *b : {&h->content, &h->cv0, &h->enc, &h->scratch, &h->hash, &h->cv1}) *b = DevBuf{};
    h->va_content = h->va_cv0 = false;
}

void hasher_destroy(chip_bao_hasher *h) {
    hasher_release_buffers(h);
    if (h->hstream) (void)hipStreamDestroy(h->hstream);
    if (h->stream) {
        stream_queue_release(h->stream);
        (void)hipStreamDestroy(h->stream);
    }
    if (h->copied) (void)hipEventDestroy(h->copied);
    delete h;
}

bool hasher_cache_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_HASHER_CACHE");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

// CHIP_HASHER_VA=0: the hasher grows by copying (grow_keep), as before round 4 (A/B)
bool hasher_va_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_HASHER_VA");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

hipError_t grow_keep(DevBuf &b, size_t need, size_t used, hipStream_t s);

// VA reserved per hasher buffer: the first reservation holds 1 GiB of content
// (or twice the first growth), its chunk CVs 1 GiB (the arena's unit); a
// buffer that outgrows its range moves once into a fresh range 4x its need
// (one device copy of the bytes so far, ~0.4 ms per GiB).  A range is never
// mapped twice (hbm_alloc.hpp), so a released hasher retires its ranges: VA
// spent grows with the bytes hashed (at most ~5x), not a flat 17 GiB each.
constexpr uint64_t HASHER_VA_CONTENT = 1ull << 30, HASHER_VA_CV = 1ull << 30;
uint64_t hasher_va_content() {
    const char *e = std::getenv("CHIP_HASHER_VA_MIB");
    const uint64_t mib = e ? std::strtoull(e, nullptr, 10) : 0;
    return mib ? mib << 20 : HASHER_VA_CONTENT;
}

// Grow a hasher buffer to `need` bytes keeping its first `used`: in place
// behind its reserved VA range (hbm::Growable) when it lives there; past the
// range, into a fresh range 4x the need (one copy after `wait_s`, whose
// kernels read the old buffer, is idle); without the VA API (or
// CHIP_HASHER_VA=0), by copying into a larger plain allocation.
hipError_t hasher_grow(DevBuf &b, chip::hbm::Growable &g, bool &in_va, size_t need, size_t used, hipStream_t copy_s,
                       hipStream_t wait_s, uint64_t reserve) {
    if (b.cap >= need) return hipSuccess;
    if ((in_va || !b.p) && hasher_va_on()) {
        hipError_t e = g.grow(need, std::max<uint64_t>(reserve, 2 * (uint64_t)need));
        if (e == hipSuccess) {
            b.p = g.va;
            b.cap = g.mapped;
            in_va = true;
            return hipSuccess;
        }
        (void)hipGetLastError();
        if (!in_va) {
            g.release();  // a first growth that failed part way: its pieces and range go
        } else {
            chip::hbm::Growable ng;  // past the range: a fresh one, 4x the need
            e = ng.grow(need, 4 * (uint64_t)need);
            if (e == hipSuccess) e = hipStreamSynchronize(wait_s);
            if (e == hipSuccess && used) e = hipMemcpyAsync(ng.va, b.p, used, hipMemcpyDeviceToDevice, copy_s);
            if (e == hipSuccess) e = hipStreamSynchronize(copy_s);
            if (e == hipSuccess) {
                g.release();
                g = std::move(ng);
                b.p = g.va;
                b.cap = g.mapped;
                return hipSuccess;
            }
            (void)hipGetLastError();
            (void)hipStreamSynchronize(copy_s);
            ng.release();
        }
    }
    hipError_t e = hipStreamSynchronize(wait_s);
    if (e != hipSuccess) return e;
    if (!in_va) return grow_keep(b, need, used, copy_s);
    DevBuf nb;  // no fresh range to be had: one copy into plain memory
    if ((e = grow_keep(nb, std::max(need, 2 * (size_t)g.mapped), 0, copy_s)) != hipSuccess) return e;
    if (used && (e = hipMemcpyAsync(nb.p, b.p, used, hipMemcpyDeviceToDevice, copy_s)) == hipSuccess)
        e = hipStreamSynchronize(copy_s);
    if (e != hipSuccess) {
        (void)hipFree(nb.p);
        return e;
    }
    g.release();
    in_va = false;
    b = nb;
    nb.p = nullptr;
    return hipSuccess;
}

// grow keeping the first `used` bytes (geometric, so appends are amortised O(1))
hipError_t grow_keep(DevBuf &b, size_t need, size_t used, hipStream_t s) {
    if (b.cap >= need) return hipSuccess;
    size_t cap = std::max(need, 2 * b.cap);
    cap = (cap + 4095) & ~size_t(4095);
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) return e;
    if (used) {
        e = hipMemcpyAsync(p, b.p, used, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
    }
    if (b.p) (void)hipFree(b.p);
    b.p = p;
    b.cap = cap;
    return hipSuccess;
}

}  // namespace

extern "C" {

int chip_bao_hasher_new(chip_bao_hasher **out) {
    if (!out) return CHIP_ERR_INVALID_ARG;
    Ctx *c;
    int st = ctx_get(&c);  // device check + hipSetDevice
    if (st != CHIP_OK) return st;
    {  // the most recently freed hasher's streams and grown buffers that lived on this device
        std::lock_guard<std::mutex> lk(g_hasher_spare_mu);
        for (size_t i = g_hasher_spares.size(); i-- > 0;) {
            chip_bao_hasher *s = g_hasher_spares[i];
            if (s->dev == c->dev && s->va_content_bytes == hasher_va_content()) {
                g_hasher_spares.erase(g_hasher_spares.begin() + (std::ptrdiff_t)i);
                *out = s;
                return CHIP_OK;
            }
        }
    }
    auto *h = new chip_bao_hasher();
    h->va_content_bytes = hasher_va_content();
    h->dev = c->dev;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->hstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->copied, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (h->copied) (void)hipEventDestroy(h->copied);
        if (h->hstream) (void)hipStreamDestroy(h->hstream);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        set_device_error(e);
        return CHIP_ERR_DEVICE;
    }
    *out = h;
    return CHIP_OK;
}

int chip_bao_hasher_update(chip_bao_hasher *h, const uint8_t *buf, uint64_t n) {
    if (!h || (!buf && n)) return CHIP_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->finalized) return CHIP_ERR_INVALID_ARG;
    if (!n) return CHIP_OK;
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    CHIP_HIP(hasher_grow(h->content, h->gcontent, h->va_content, h->len + n, h->len, h->stream, h->hstream,
                         h->va_content_bytes));
    // the caller may reuse buf on return: a staged copy is done with it already, a direct one
    // (pinned buf) is waited for on every return path below, the error paths included
    struct SyncDirect {
        hipStream_t s;
        bool on;
        ~SyncDirect() {
            if (on) (void)hipStreamSynchronize(s);
        }
    } sync_direct{h->stream, false};
    CHIP_HIP(h2d(c->stage, static_cast<uint8_t *>(h->content.p) + h->len, buf, n, h->stream));
    sync_direct.on = !staged(buf, n);
    h->len += n;
    // units u with bytes past them ((u + 1) * 64 KiB < len): full chunks, none of them the last;
    // hashed on the second stream once their bytes have landed, so the copies never wait for it.
    // One launch per 32 MiB of new units (512): an event, a stream wait and a launch per 4 MiB
    // append cost the appends 14 % (profiles/r6t); finalize hashes what is left.
    const uint64_t ready = (h->len - 1) / 65536;
    if (hasher_batch_units() && ready >= h->units + hasher_batch_units()) {
        CHIP_HIP(hasher_grow(h->cv0, h->gcv0, h->va_cv0, std::max<uint64_t>(ready * 64 * 32, 1 << 20),
                             h->units * 64 * 32, h->hstream, h->hstream, HASHER_VA_CV));
        CHIP_HIP(hipEventRecord(h->copied, h->stream));
        CHIP_HIP(hipStreamWaitEvent(h->hstream, h->copied, 0));
        CHIP_HIP(hasher_chunks_dev(static_cast<const uint8_t *>(h->content.p), h->len, h->units * 64, ready * 64,
                                   static_cast<uint8_t *>(h->cv0.p), h->hstream));
        h->units = ready;
    }
    if (sync_direct.on) {
        sync_direct.on = false;
        CHIP_HIP(hipStreamSynchronize(h->stream));
    }
    return CHIP_OK;
}

int chip_bao_hasher_finalize(chip_bao_hasher *h, uint8_t hash[CHIP_HASH_LEN]) {
    if (!h || !hash) return CHIP_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->finalized) {
        Ctx *c;
        int st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        const uint64_t n = h->len;
        h->enc_len = bao_encoded_len(n);
        CHIP_HIP(hasher_grow(h->content, h->gcontent, h->va_content, 16, h->len, h->stream, h->hstream,
                             h->va_content_bytes));
        CHIP_HIP(grow(h->enc, h->enc_len));
        CHIP_HIP(grow(h->hash, 32));
        if (h->units == 0) {  // under 64 KiB + 1 byte in all: the batch path in one go
            CHIP_HIP(grow(h->scratch, bao_scratch_len(n, 1)));
            CHIP_HIP(bao_encode_dev(static_cast<const uint8_t *>(h->content.p), 0, n, 1,
                                    static_cast<uint8_t *>(h->enc.p), 0, static_cast<uint8_t *>(h->hash.p),
                                    h->scratch.p, h->stream));
        } else {  // only the last chunks are hashed here
            const uint64_t N = (n + 1023) / 1024;
            CHIP_HIP(hipStreamSynchronize(h->hstream));  // update()'s chunk CVs are in cv0
            CHIP_HIP(hasher_grow(h->cv0, h->gcv0, h->va_cv0, N * 32, h->units * 64 * 32, h->stream, h->hstream,
                                 HASHER_VA_CV));
            CHIP_HIP(grow(h->cv1, (N + 1) / 2 * 32));
            CHIP_HIP(hasher_finish_dev(static_cast<const uint8_t *>(h->content.p), n, h->units * 64,
                                       static_cast<uint8_t *>(h->cv0.p), static_cast<uint8_t *>(h->cv1.p),
                                       static_cast<uint8_t *>(h->enc.p), static_cast<uint8_t *>(h->hash.p),
                                       h->stream));
        }
        CHIP_HIP(hipMemcpyAsync(h->h, h->hash.p, 32, hipMemcpyDeviceToHost, h->stream));
        CHIP_HIP(hipStreamSynchronize(h->stream));
        h->finalized = true;
    }
    std::memcpy(hash, h->h, 32);
    return CHIP_OK;
}

uint64_t chip_bao_hasher_len(chip_bao_hasher *h) {
    if (!h) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    return h->len;
}

int chip_bao_hasher_read_all(chip_bao_hasher *h, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!h || !out_len) return CHIP_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (!h->finalized) return CHIP_ERR_INVALID_ARG;
    *out_len = h->enc_len;
    if (out_cap < h->enc_len || !out) return CHIP_ERR_BUFFER_TOO_SMALL;
    Ctx *c;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    CHIP_HIP(d2h(c->stage, out, h->enc.p, h->enc_len, h->stream));
    CHIP_HIP(hipStreamSynchronize(h->stream));
    return CHIP_OK;
}

void chip_bao_hasher_free(chip_bao_hasher *h) {
    if (!h) return;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        if (h->hstream) (void)hipStreamSynchronize(h->hstream);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        if (hasher_cache_on()) {  // park it, emptied, for the next chip_bao_hasher_new
            std::lock_guard<std::mutex> sk(g_hasher_spare_mu);
            if (g_hasher_spares.size() < HASHER_PARK_COUNT) {
                uint64_t parked = 0;
                for (const chip_bao_hasher *s : g_hasher_spares) parked += hasher_bytes(s);
                if (parked + hasher_bytes(h) > hasher_park_bytes()) hasher_release_buffers(h);  // streams only
                h->len = h->enc_len = h->units = 0;
                h->finalized = false;
                std::memset(h->h, 0, sizeof h->h);
                g_hasher_spares.push_back(h);
                return;
            }
        }
    }
    hasher_destroy(h);
}

uint64_t chip_bao_hasher_drop_cache(void) {
    std::vector<chip_bao_hasher *> all;
    {
        std::lock_guard<std::mutex> sk(g_hasher_spare_mu);
        all.swap(g_hasher_spares);
    }
    uint64_t freed = 0;
    for (chip_bao_hasher *h : all) {  // parked hashers: their work was synchronised when they were freed
        freed += hasher_bytes(h);
        (void)hipSetDevice(h->dev);
        hasher_destroy(h);
    }
    if (!all.empty()) (void)use_device();
    return freed;
}

uint64_t chip_bao_hasher_cached_bytes(void) {
    std::lock_guard<std::mutex> sk(g_hasher_spare_mu);
    uint64_t s = 0;
    for (const chip_bao_hasher *h : g_hasher_spares) s += hasher_bytes(h);
    return s;
}

}  // extern "C"
