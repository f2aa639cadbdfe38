// api_context.cpp — device selection, the per-thread context (stream,
// grow-only device scratch, pinned arena for the few-byte copies of a
// call), library info, size helpers and batch-buffer allocation.  Shared
// declarations: api_common.hpp.
#include <mutex>

#include "api_common.hpp"

namespace chip {
namespace api {

std::once_flag g_dev_once;
std::atomic<int> g_device{-1};  // the process's device (one GPU per process, see chip_init)
std::atomic<int> g_cus{0};
int g_dev_status = CHIP_ERR_NO_DEVICE;
thread_local std::string t_last_err;

bool is_gfx950(int d, int *cus) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) return false;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return false;
    if (cus) *cus = prop.multiProcessorCount;
    return true;
}

// Default device: the caller's current HIP device when it is a gfx950 (so a
// process that selected its GPU first, e.g. torch.cuda.set_device(local_rank),
// is followed), else the first gfx950.  chip_init(d) selects explicitly.
void init_device_once() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        t_last_err = "no HIP device visible";
        return;
    }
    int cur = -1, cus = 0;
    if (hipGetDevice(&cur) == hipSuccess && cur >= 0 && cur < n && is_gfx950(cur, &cus)) {
        g_device = cur;
        g_cus = cus;
        g_dev_status = CHIP_OK;
        return;
    }
    for (int d = 0; d < n; ++d)
        if (is_gfx950(d, &cus)) {
            g_device = d;
            g_cus = cus;
            g_dev_status = CHIP_OK;
            return;
        }
    t_last_err = "no gfx950 device visible";
}

void Staging::release() {
    for (int k = 0; k < R; ++k) {
        if (ev[k]) (void)hipEventDestroy(ev[k]);
        ev[k] = nullptr;
        armed[k] = false;
    }
    if (ring) (void)hipHostFree(ring);
    ring = nullptr;
}

void Ctx::release() {
    stage.release();
    if (hs.p) (void)hipHostFree(hs.p);
    hs = DevBuf{};
    if (ev_km) (void)hipEventDestroy(ev_km);
    ev_km = nullptr;
    for (DevBuf *b : {&hin, &hout}) {
        if (b->p) (void)hipHostFree(b->p);
        *b = DevBuf{};
    }
    hs_used = 0;
    hs_out.clear();
    // best effort (at process teardown the runtime may already be gone)
    for (DevBuf *b : {&in, &mid, &out, &scratch, &small, &x1, &x2, &flags}) {
        if (b->p) (void)hipFree(b->p);
        *b = DevBuf{};
    }
    if (stream) {
        (void)hipStreamSynchronize(stream);
        stream_queue_release(stream);
        (void)hipStreamDestroy(stream);
    }
    stream = nullptr;
    for (Slot &sl : slots) {
        for (DevBuf *b : {&sl.in, &sl.mid, &sl.out, &sl.hash, &sl.scratch, &sl.nodes, &sl.sin})
            if (b->p) (void)hipFree(b->p);
        for (DevBuf *b : {&sl.stage, &sl.hnodes})
            if (b->p) (void)hipHostFree(b->p);
        if (sl.stream) {
            (void)hipStreamSynchronize(sl.stream);
            stream_queue_release(sl.stream);
            (void)hipStreamDestroy(sl.stream);
        }
    }
    slots.clear();
    ready = false;
}

namespace {
thread_local Ctx t_ctx;
}  // namespace

hipError_t grow(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return hipSuccess;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.cap = 0;
    }
    size_t cap = bytes + (bytes >> 3);  // grow-only with headroom
    cap = (cap + 255) & ~size_t(255);
    hipError_t e = hipMalloc(&b.p, cap);
    if (e != hipSuccess) return e;
    b.cap = cap;
    return hipSuccess;
}

hipError_t grow_pinned(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return hipSuccess;
    if (b.p) {
        hipError_t e = hipHostFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.cap = 0;
    }
    size_t cap = ((bytes + (bytes >> 3)) + 4095) & ~size_t(4095);
    hipError_t e = hipHostMalloc(&b.p, cap, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    b.cap = cap;
    return hipSuccess;
}

}  // namespace api

using namespace api;

int ensure_device() {
    std::call_once(g_dev_once, init_device_once);
    return g_dev_status;
}

void set_device_error(hipError_t e) { t_last_err = hipGetErrorString(e); }

int num_cus() { return g_cus > 0 ? g_cus.load() : 256; }

int selected_device() { return g_device; }

int use_device() {
    int st = ensure_device();
    if (st != CHIP_OK) return st;
    hipError_t e = hipSetDevice(g_device);
    if (e != hipSuccess) {
        set_device_error(e);
        return CHIP_ERR_DEVICE;
    }
    return CHIP_OK;
}

namespace api {

int ctx_get(Ctx **out) {
    int st = ensure_device();
    if (st != CHIP_OK) return st;
    Ctx &c = t_ctx;
    const int dev = g_device;
    if (c.ready && c.dev != dev) {  // the process switched devices (chip_init): drop the old context
        (void)hipSetDevice(c.dev);
        c.release();
    }
    CHIP_HIP(hipSetDevice(dev));
    if (!c.ready) {
        CHIP_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        c.dev = dev;
        c.ready = true;
    }
    if (c.hs_used) {  // an earlier call returned early: let its copies land, drop its outputs
        c.hs_out.clear();
        c.hs_used = 0;
        CHIP_HIP(hipStreamSynchronize(c.stream));
    }
    *out = &c;
    return CHIP_OK;
}

// ---- few-byte copies of a single-object call ------------------------------
// hipMemcpyAsync on pageable memory costs ~22 us of API time per call, even
// for 4 bytes (profiles/r4c: the runtime stages and waits), which dominated
// small objects' latency.  Hashes, status words and node flags therefore go
// through a pinned per-context arena: small_h2d copies the bytes in at once,
// small_d2h lands them there and small_sync (the call's stream
// synchronisation) hands them to their destinations.
constexpr size_t kHostSmall = size_t(64) << 10;

hipError_t small_h2d(Ctx *c, void *ddst, const void *src, size_t n) {
    if (!n) return hipSuccess;
    const size_t need = (n + 15) & ~size_t(15);
    if (!c->hs.p) {
        hipError_t e = grow_pinned(c->hs, kHostSmall);
        if (e != hipSuccess) return e;
    }
    if (c->hs_used + need > c->hs.cap) return hipMemcpyAsync(ddst, src, n, hipMemcpyHostToDevice, c->stream);
    uint8_t *p = static_cast<uint8_t *>(c->hs.p) + c->hs_used;
    c->hs_used += need;
    std::memcpy(p, src, n);
    return hipMemcpyAsync(ddst, p, n, hipMemcpyHostToDevice, c->stream);
}

// `dst` receives the n bytes at the next small_sync (or d2h_sync)
hipError_t small_d2h(Ctx *c, void *dst, const void *dsrc, size_t n) {
    if (!n) return hipSuccess;
    const size_t need = (n + 15) & ~size_t(15);
    if (!c->hs.p) {
        hipError_t e = grow_pinned(c->hs, kHostSmall);
        if (e != hipSuccess) return e;
    }
    if (c->hs_used + need > c->hs.cap) return hipMemcpyAsync(dst, dsrc, n, hipMemcpyDeviceToHost, c->stream);
    uint8_t *p = static_cast<uint8_t *>(c->hs.p) + c->hs_used;
    c->hs_used += need;
    c->hs_out.push_back({dst, p, n});
    return hipMemcpyAsync(p, dsrc, n, hipMemcpyDeviceToHost, c->stream);
}

void small_deliver(Ctx *c) {
    for (const Ctx::HsOut &o : c->hs_out) std::memcpy(o.dst, o.src, o.n);
    c->hs_out.clear();
    c->hs_used = 0;
}

// the call's stream work is done and its small outputs delivered
hipError_t small_sync(Ctx *c) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) small_deliver(c);
    return e;
}

}  // namespace api
}  // namespace chip

using namespace chip;
using namespace chip::api;

extern "C" {

int chip_abi_version(void) { return CHIP_ABI_VERSION; }

const char *chip_strerror(int st) {
    switch (st) {
        case CHIP_OK: return "ok";
        case CHIP_ERR_INVALID_ARG: return "invalid argument";
        case CHIP_ERR_BUFFER_TOO_SMALL: return "output buffer too small";
        case CHIP_ERR_UNEVEN_ZFEC_CHUNKS: return "Input bytes must divide evenly over number of zfec chunks.";
        case CHIP_ERR_HASH_DECODE: return "Hash must be 32 bytes long.";
        case CHIP_ERR_BAO_HASH_MISMATCH: return "bao decode error: hash mismatch";
        case CHIP_ERR_BAO_TRUNCATED: return "bao decode error: encoding truncated";
        case CHIP_ERR_ZFEC: return "zfec error";
        case CHIP_ERR_ENCODE_ZFEC_PADDING: return "Padding from Zfec should always be zero.";
        case CHIP_ERR_ENCODE_INVALID_CHUNK_LENGTH: return "Chunk length should be as calculated.";
        case CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT: return "Verifiable slice count should be evenly divisible by 8.";
        case CHIP_ERR_UNSUPPORTED_FORMAT: return "unsupported format";
        case CHIP_ERR_UNNECESSARY_SCRUB: return "Data does not need to be scrubbed.";
        case CHIP_ERR_SCRUBBED_PADDING_MISMATCH: return "Scrubbed padding should remain the same.";
        case CHIP_ERR_SCRUBBED_LENGTH_MISMATCH: return "Mismatch between scrubbed data length and input length";
        case CHIP_ERR_INVALID_SCRUBBED_HASH: return "Scrubbed hash is not equal to original hash.";
        case CHIP_ERR_SNAP: return "snappy framing error";
        case CHIP_ERR_ECIES: return "ecies error";
        case CHIP_ERR_SECP256K1: return "secp256k1 error (key, message or signature)";
        case CHIP_ERR_INVALID_HEADER_LENGTH: return "Invalid header length calculation";
        case CHIP_ERR_INVALID_MAGIC: return "File header lacks Carbonado magic number and may not be a proper Carbonado file.";
        case CHIP_ERR_NO_DEVICE: return "no usable gfx950 device";
        case CHIP_ERR_DEVICE: return "HIP runtime error";
        default: return "unknown status";
    }
}

int chip_init(int device) {
    int st = ensure_device();
    if (st != CHIP_OK) return st;
    if (device >= 0) {
        int n = 0, cus = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || device >= n || !is_gfx950(device, &cus)) {
            t_last_err = "device " + std::to_string(device) + " is not a visible gfx950";
            return CHIP_ERR_NO_DEVICE;
        }
        g_cus = cus;
        g_device = device;
    }
    Ctx *c;
    return ctx_get(&c);
}

const char *chip_last_device_error(void) { return t_last_err.c_str(); }

int chip_calc_padding_len(uint64_t input_len, uint32_t k, uint32_t *padding, uint32_t *chunk_len) {
    if (!padding || !chunk_len || k == 0) return CHIP_ERR_INVALID_ARG;
    uint64_t C;
    calc_pad(input_len, k, padding, &C);
    *chunk_len = (uint32_t)C;
    return CHIP_OK;
}

uint64_t chip_zfec_encoded_len(uint64_t n, uint32_t k, uint32_t m) {
    if (k == 0) return 0;
    uint32_t pad;
    uint64_t C;
    calc_pad(n, k, &pad, &C);
    return (uint64_t)m * C;
}

uint64_t chip_bao_encoded_len(uint64_t n) { return bao_encoded_len(n); }

uint64_t chip_encode_max_len(uint64_t n) {
    const uint64_t h = host_stage_max(CHIP_FORMAT_SNAPPY | CHIP_FORMAT_ECIES, n);  // >= n
    const uint64_t z = chip_zfec_encoded_len(h, CHIP_FEC_K, CHIP_FEC_M);
    const uint64_t big = z > h ? z : h;
    return bao_encoded_len(big);
}

uint64_t chip_snap_max_len(uint64_t n) { return host::snap_max_len(n); }

uint64_t chip_bao_scratch_len(uint64_t n, uint64_t count) { return bao_scratch_len(n, count); }

// Batch buffers.  From 1 GiB up: class-balanced memory (hbm_alloc.hpp):
// physical pieces spread over the HBM "classes" and mapped shuffled, so the
// streaming kernels never write into one class only (DESIGN.md §2, §3 K1:
// 4-of-8 encode 0.63-0.67 -> 0.77-0.78 of the roofline).  Smaller buffers,
// or CHIP_ALLOC=contiguous: physically contiguous memory
// (hipDeviceMallocContiguous), else hipMalloc.
int chip_device_alloc(uint64_t bytes, void **ptr) {
    if (!ptr) return CHIP_ERR_INVALID_ARG;
    *ptr = nullptr;
    int st = use_device();
    if (st != CHIP_OK) return st;
    void *p = nullptr;
    const size_t sz = bytes ? bytes : 1;
    const char *mode = std::getenv("CHIP_ALLOC");
    const bool balanced = !(mode && std::strcmp(mode, "contiguous") == 0);
    if (balanced && hbm_alloc(sz, &p) == hipSuccess && p) {
        *ptr = p;
        return CHIP_OK;
    }
    (void)hipGetLastError();
    p = nullptr;
    if (hipExtMallocWithFlags(&p, sz, hipDeviceMallocContiguous) != hipSuccess || !p) {
        (void)hipGetLastError();
        p = nullptr;
        CHIP_HIP(hipMalloc(&p, sz));
    }
    *ptr = p;
    return CHIP_OK;
}

int chip_device_free(void *ptr) {
    if (!ptr) return CHIP_OK;
    if (hbm_free(ptr)) return CHIP_OK;
    CHIP_HIP(hipFree(ptr));
    return CHIP_OK;
}

int chip_device_alloc_info(const void *ptr, uint32_t *classes_found, uint32_t *classes_used, double *seconds) {
    uint32_t f = 0, u = 0;
    double t = 0;
    if (!ptr || !hbm_info(ptr, &f, &u, &t)) return CHIP_ERR_INVALID_ARG;
    if (classes_found) *classes_found = f;
    if (classes_used) *classes_used = u;
    if (seconds) *seconds = t;
    return CHIP_OK;
}

int chip_stream_queue_block(void *stream, uint64_t *addr) {
    if (!addr) return CHIP_ERR_INVALID_ARG;
    int st = use_device();
    if (st != CHIP_OK) return st;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!s) {
        Ctx *c = nullptr;
        st = ctx_get(&c);
        if (st != CHIP_OK) return st;
        s = c->stream;
    }
    uint32_t *q = nullptr;
    CHIP_HIP(chip::stream_queue(s, &q));
    *addr = (uint64_t)(uintptr_t)q;
    return CHIP_OK;
}


void chip_torch_free(void *ptr, ssize_t size, int device, void *stream) {
    (void)size;
    (void)stream;
    (void)hipSetDevice(device);
    (void)chip_device_free(ptr);
}


}  // extern "C"
