// api_common.hpp — what the C-ABI translation units of libcarbonado_hip share
// (include/carbonado_hip.h).  Host-side orchestration only: argument checks
// and error mapping that mirror the reference stage functions (file:line
// cited per entry point), staging of host buffers into per-thread device
// scratch, and the encode()/decode() glue.  Every byte of shard/stream data is
// produced by the HIP kernels in zfec_kernels.hip, bao_kernels.hip,
// fused_kernels.hip and small_kernels.hip; there is no CPU compute path for
// zfec or bao.  The snappy/ECIES stages that the reference runs before zfec
// (and after it on decode) are host stages by design (host_stages.cpp).
//
// The entry points, by concern:
//   api_context.cpp    device selection, the per-thread context, small
//                      copies, library info, sizes, batch-buffer allocation
//   api_host_copy.cpp  host <-> HBM copies (pinned ring, copy threads, NUMA)
//   api_plans.cpp      zfec plans, encode() at Zfec|Bao on the device, bao
//                      and slice geometry, EncodeInfo, host-stage glue
//   api_stages.cpp     the stage functions and the device-resident batches
//   api_scrub.cpp      verify_slice / extract_slice / scrub (single, batch)
//   api_encode.cpp     encode() from host memory (single, host batch)
//   api_decode.cpp     decode() from host memory (single, host batch)
//   api_hasher.cpp     the streaming BaoHasher
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "chip_internal.hpp"
#include "gf256.hpp"
#include "host_stages.hpp"

#define CHIP_HIP(expr)                                  \
    do {                                                \
        hipError_t e__ = (expr);                        \
        if (e__ != hipSuccess) {                        \
            ::chip::set_device_error(e__);              \
            return CHIP_ERR_DEVICE;                     \
        }                                               \
    } while (0)

namespace chip {
namespace api {

// ---- device and per-thread context (api_context.cpp) ----------------------
extern std::atomic<int> g_device;  // the process's device (one GPU per process, see chip_init)
extern std::atomic<int> g_cus;
extern thread_local std::string t_last_err;

bool is_gfx950(int d, int *cus);

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

// one pipeline slot of chip_encode_host_batch: its own stream and buffers
// (`stage` is pinned host memory holding the host-stage output of a slice)
struct Slot {
    hipStream_t stream = nullptr;
    DevBuf in, mid, out, hash, scratch, nodes, sin;  // sin: data regions taken from host rows
    DevBuf stage, hnodes;  // pinned
};

// Pinned ring for copies between PAGEABLE host memory and HBM (see h2d/d2h).
struct Staging {
    static constexpr int R = 4;
    static constexpr size_t PIECE = size_t(4) << 20;
    uint8_t *ring = nullptr;
    hipEvent_t ev[R] = {};
    bool armed[R] = {};
    unsigned next = 0;  // ring slot of the next piece (rotates across calls)
    void release();
};

struct Ctx {
    bool ready = false;
    int dev = -1;  // device the stream and buffers live on
    hipStream_t stream = nullptr;
    DevBuf in, mid, out, scratch, small, x1, x2, flags;
    DevBuf hin, hout;  // pinned, NUMA-local: a single object's zero-copy input / outputs (api_single.cpp)
    hipEvent_t ev_km = nullptr;  // api_single.cpp: the parity kernel of a single encode done
    std::vector<Slot> slots;
    Staging stage;
    // pinned arena for the few-byte copies of a call (hashes, status words,
    // node flags): see small_h2d / small_d2h / small_sync
    DevBuf hs;
    size_t hs_used = 0;
    struct HsOut {
        void *dst;
        const uint8_t *src;
        size_t n;
    };
    std::vector<HsOut> hs_out;
    void release();
    ~Ctx() { release(); }
};

hipError_t grow(DevBuf &b, size_t bytes);         // grow-only device buffer (contents dropped)
hipError_t grow_pinned(DevBuf &b, size_t bytes);  // the same, pinned host memory
// pinned host memory on the GPU's NUMA node (api_host_copy.cpp), for buffers
// the kernels read or write over PCIe themselves (zero-copy)
hipError_t grow_pinned_local(DevBuf &b, size_t bytes, unsigned flags = hipHostMallocDefault);
// the calling thread's context on the process's device (created on first use)
int ctx_get(Ctx **out);
// few-byte copies of a call through the context's pinned arena; `dst` of a
// small_d2h receives its bytes at the next small_sync
hipError_t small_h2d(Ctx *c, void *ddst, const void *src, size_t n);
hipError_t small_d2h(Ctx *c, void *dst, const void *dsrc, size_t n);
hipError_t small_sync(Ctx *c);

// ---- host <-> HBM copies (api_host_copy.cpp) --------------------------------
bool host_pinned(const void *p);
bool staged(const void *host, size_t n);  // pageable (or CHIP_HOST_COPY=staged): through the pinned ring
// host -> HBM on s; on return `src` may be reused
hipError_t h2d(Staging &sg, void *dst, const void *src, size_t n, hipStream_t s);
// HBM -> host after the work already on s; returns when `dst` holds the bytes
hipError_t d2h(Staging &sg, void *dst, const void *src, size_t n, hipStream_t s);
// d2h in two halves: begin enqueues (the first ring pieces' DMA), end copies
// out and returns when `dst` holds the bytes; the caller may work between
// them (nothing else may use the ring meanwhile).
struct D2h {
    void *dst = nullptr;
    const void *src = nullptr;
    size_t n = 0;
    hipStream_t s = nullptr;
    size_t np = 0;
    unsigned base = 0;
    bool direct = false;
};
hipError_t d2h_begin(Staging &sg, D2h &t, void *dst, const void *src, size_t n, hipStream_t s);
// advise the 2 MiB-aligned interior of a host output of >= 4 MiB onto
// transparent huge pages before the host threads first write it (d2h does
// so for pageable destinations; CHIP_OUT_THP=0 turns it off)
void advise_huge(void *p, uint64_t n);
hipError_t d2h_issue(Staging &sg, const D2h &t, size_t j);
hipError_t d2h_end(Staging &sg, const D2h &t);

// Pitch of the device rows the library lays out itself (slot buffers): a
// multiple of 256 B, so every row's shards start on a 128-B line.  With
// 16-B rows each 128-B piece a wave loads straddles two lines and K13 /
// K1 fetch 1.21x the input bytes (tools/k13_fetch, profiles/r10c_session).
inline uint64_t row_pitch(uint64_t n) { return (n + 255) / 256 * 256; }

// ---- plans and geometry (api_plans.cpp) ------------------------------------
int env_int(const char *name, int dflt);
bool valid_km(uint32_t k, uint32_t m);
void calc_pad(uint64_t n, uint32_t k, uint32_t *pad, uint64_t *C);  // utils.rs:47-58, k generalised
// rows 0..k-1 copied, k..m-1 computed (aliased: in place, parity rows only)
GfPlan encode_plan(uint32_t k, uint32_t m, uint64_t C, const std::vector<uint8_t> &enc, bool aliased = false);
// whether zfec_bao_dev writes the streams with K13, which takes any 8-B
// aligned stream base (its line stores split each chunk at the memory lines
// wherever they fall); KS and the two-kernel path want 16-B aligned rows
bool zfec_bao_any8(uint64_t C, uint64_t count);
// where the library's own slot rows put a K13 stream (CHIP_STREAM_OFFSET, a
// multiple of 8 below 256; default 56: every chunk and node on a 64-B boundary)
uint64_t stream_offset();
// encode() at Zfec|Bao of device-resident objects (K13, or KS for small ones)
hipError_t zfec_bao_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                        uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch, hipStream_t s);
int decode_plan(uint32_t k, uint32_t m, uint64_t C, const std::vector<uint32_t> &sel,
                const std::vector<uint64_t> &slot_off, GfPlan *out);
int select_shares(uint32_t k, uint32_t m, const uint32_t *idx, uint32_t nshares, std::vector<uint32_t> *sel_pos);
uint64_t n_chunks_of(uint64_t n);
int ceil_log2_u64(uint64_t x);
void slice_chunks(uint64_t n, uint64_t start, uint64_t len, uint64_t *c0, uint64_t *c1);
struct SliceNode {
    bool parent;
    uint64_t off, len, index;  // stream offset, bytes, chunk index or parent index (stream order)
};
void slice_nodes(uint64_t n, uint64_t c0, uint64_t c1, std::vector<SliceNode> *out);
int encode_info_for(uint8_t format, uint64_t input_len, uint64_t cur, uint64_t bc, uint64_t be,
                    chip_encode_info *inf, uint64_t *zlen, uint64_t *final_len);
bool has_host_stages(uint8_t format);

// grow-only, uninitialised host scratch (std::vector::resize would zero-fill
// and page-fault 16 MiB per object)
struct Scratch {
    std::unique_ptr<uint8_t[]> p;
    size_t cap = 0;
    uint8_t *get(size_t n) {
        if (n > cap) {
            p.reset(new uint8_t[n]);
            cap = n;
        }
        return p.get();
    }
};

bool stream_encrypt_on();
uint64_t host_stage_max(uint8_t format, uint64_t n);
int host_stages_into(uint8_t format, const uint8_t *pk, uint64_t pklen, const uint8_t *eph, const uint8_t *nonce,
                     const uint8_t *in, uint64_t n, uint8_t *dst, uint64_t cap, Scratch &tmp,
                     uint64_t *len, uint64_t *bc, uint64_t *be, const host::ChunkSink *sink = nullptr,
                     uint64_t *filled = nullptr, const host::EciesKey *prepared = nullptr, bool par = false);

// ---- one object from host memory on KM (api_single.cpp) ---------------------
// CHIP_SINGLE_TRACE=1: the host-side phases of each call to stderr (us)
struct Trace {
    const char *what;
    bool on;
    std::chrono::steady_clock::time_point t0, last;
    explicit Trace(const char *w) : what(w), on(enabled()) {
        if (on) t0 = last = std::chrono::steady_clock::now();
    }
    static bool enabled() {
        static const bool e = [] {
            const char *v = std::getenv("CHIP_SINGLE_TRACE");
            return v && v[0] == '1';
        }();
        return e;
    }
    void mark(const char *phase) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[single %s] %-12s +%7.1f us (%7.1f)\n", what, phase,
                     std::chrono::duration<double, std::micro>(now - last).count(),
                     std::chrono::duration<double, std::micro>(now - t0).count());
        last = now;
    }
};

// encode() at Zfec|Bao (C > 0: the zfec shard length) or bao of the content
// (C == 0) of cur_n bytes at `cur` into out[0, final_len) and the root hash,
// with the split copy-back: the host writes the stream's header and the chunks
// it already holds (the content / data shards) while the device hashes; only
// the parity region and the parent nodes cross PCIe.  km_ok() must hold.
// `cur` may be c->hin itself (the host stages' output written there, hin
// already grown to cur_n + 16): the copy into pinned memory is then skipped.
int single_encode_km(Ctx *c, const uint8_t *cur, uint64_t cur_n, uint64_t C, uint64_t final_len, uint8_t *out,
                     uint8_t hash[32]);
// encoding::zfec 4-of-8 of one object (n > 0 bytes, shard length C) into
// out[0, 8 C): the host writes the data shards (the zero-padded input) while
// parity_kernel<1> reads the input from pinned memory and writes the parity
// shards into pinned memory (zero-copy), copied out after.
int single_zfec_encode_zc(Ctx *c, const uint8_t *in, uint64_t n, uint64_t C, uint8_t *out);
// zfec decode of one object from k shares (shares[s] holds share sel[s], C
// bytes): the host copies the shares into pinned memory, the decode kernel
// reads them there and writes the k data shards there (zero-copy), and the
// first olen bytes are copied to dst.  `meanwhile` (optional) runs on the host
// while the kernel works.
int single_zfec_decode_zc(Ctx *c, uint32_t k, uint32_t m, const uint8_t *const *shares,
                          const std::vector<uint32_t> &sel, uint64_t C, uint8_t *dst, uint64_t olen,
                          const std::function<void()> &meanwhile = {});
// decode of one bao stream `in` (len bytes, content n, every node verified on
// the device by KM) with the content bytes [0, olen) gathered from `in` by the
// host meanwhile, into dst; on a mismatch dst is wiped and the status
// returned.  km_ok() must hold.
// `meanwhile` (optional) runs on the host beside the gather (a pool task of
// its own when the gather takes several) or after it, before the wait;
// `gathered` (optional) after both, still before the wait: it may read
// dst[0, olen), which is unverified until the call returns CHIP_OK.
int single_decode_km(Ctx *c, const uint8_t *in, uint64_t len, uint64_t n, const uint8_t *hash, uint8_t *dst,
                     uint64_t olen, const std::function<void()> &meanwhile = {},
                     const std::function<void()> &gathered = {});

// K1 reads and writes 16-B vectors and its tail load relies on 16-B aligned
// shard addresses (zfec_device.hpp load16_masked).
inline bool misaligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) != 0; }
int zfec_decode_device(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                       const std::vector<uint64_t> &slot_off, const std::vector<uint32_t> &sel, uint64_t C,
                       uint64_t count, uint8_t *d_out, uint64_t out_stride, hipStream_t s);
bool bao_content_len(uint64_t len, uint64_t *n);
int bao_encode_ctx(Ctx *c, const uint8_t *d_in, uint64_t n, bool want_stream, uint8_t hash[32]);
int bao_decode_ctx(Ctx *c, const uint8_t *d_enc, uint64_t len, uint64_t n, const uint8_t *hash, uint8_t *d_dst,
                   uint64_t out_limit = ~0ull, uint32_t *deferred = nullptr);
int bao_header(const uint8_t *enc, uint64_t len, uint64_t *n);
int node_check_ctx(Ctx *c, uint64_t n, const uint8_t *hash, std::vector<uint8_t> *cf, std::vector<uint8_t> *pf);
bool slice_ok(uint64_t n, uint64_t c0, uint64_t c1, const std::vector<uint8_t> &cf, const std::vector<uint8_t> &pf);
int scrub_repair_enqueue(Ctx *c, const uint8_t *d_stream, uint64_t n, uint64_t len, const std::vector<uint32_t> &good,
                         uint32_t padding, uint64_t C, uint8_t *d_dst, uint8_t *d_h2);

// A zfec batch: one launch (the dynamic run queue balances the XCDs inside it).
template <typename F>  // launch(o0, cnt, stream) -> hipError_t, objects [o0, o0 + cnt)
hipError_t zf_run(uint64_t count, hipStream_t s, F launch) {
    return launch(0, count, s);
}

}  // namespace api
}  // namespace chip
