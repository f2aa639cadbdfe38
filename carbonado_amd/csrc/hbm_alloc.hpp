// hbm_alloc.hpp — class-balanced HBM allocator for batch buffers (gfx950).
//
// Why: MI355X device memory falls into "classes" that each cover several
// GiB of physical address space (tools/hbm_partition, hbm_interleave;
// DESIGN.md §3).  Streaming writes that stay inside one class run at
// ~5.4 TB/s; the same writes spread over two classes at ~6.9-7.1 TB/s
// (reads: 6.2 vs 6.45).  A multi-GiB hipMalloc comes from one physically
// contiguous range, often a single class, and the 1:2 read:write zfec
// encode over it ran at 0.63-0.67 of the 8 TB/s peak whatever the kernel's
// schedule; over memory whose pieces are spread across the classes it ran
// at 0.75-0.79 (tools/alloc_probe).
//
// How: physical memory in PIECE-sized handles (hipMemCreate), a few more
// than asked for; the handles are mapped once behind a scratch VA range,
// classified in GROUPs of consecutive pieces by timing pairwise writes (XCDs
// 0-3 write group a while XCDs 4-7 write group b: a pair much faster than a
// group with itself lies in two classes), groups are chosen round-robin over
// the classes, and the chosen pieces are mapped in a shuffled order behind a
// fresh VA range: every window of a few hundred MiB of the buffer then
// touches every class.  The scratch mapping is removed and the unchosen
// pieces are released.
//
// VA ranges are carved from a reserved arena and NEVER mapped twice: on
// ROCm 7.2 a VA range that had been mapped before (by hipMalloc, or by
// hipMemMap to other handles) and is mapped again read stale translations
// (outputs differed, tools/alloc_probe "same VA").  The arena is 4 TiB of
// VA; exhausting it falls back to a new reservation.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <map>
#include <mutex>
#include <random>
#include <vector>

namespace chip {
namespace hbm {

constexpr uint64_t MiB = 1ull << 20;
constexpr uint64_t PIECE = 8 * MiB;    // physical handle size
constexpr uint64_t GROUP = 1024 * MiB; // classification unit: 128 consecutive pieces
constexpr uint64_t PIECES_PER_GROUP = GROUP / PIECE;
constexpr uint64_t MIN_BYTES = 1024 * MiB;  // smaller buffers: plain allocations
constexpr int MAX_CLASSES = 8;

__device__ __forceinline__ uint32_t pair_xcc() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }

// XCDs 0-3 write `a`, XCDs 4-7 write `b` (each XCD a quarter of `bytes`),
// 16-B nontemporal stores in 256 KiB runs, 2 workgroups/CU.
static __global__ __launch_bounds__(256) void pair_write_kernel(uint8_t *a, uint8_t *b, uint64_t bytes) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    constexpr uint64_t RUN = 256 << 10;
    const uint32_t x = pair_xcc();
    const uint32_t g = gridDim.x / 8, w = blockIdx.x / 8;
    uint8_t *reg = (x < 4 ? a : b) + (x & 3) * (bytes / 4);
    const uint64_t runs = bytes / 4 / RUN;
    const v4 val = {blockIdx.x, threadIdx.x, 0x5a5a5a5au, 0u};
    for (uint64_t r = w; r < runs; r += g) {
        uint8_t *p = reg + r * RUN + threadIdx.x * 16;
#pragma unroll 4
        for (int i = 0; i < (int)(RUN / 4096); ++i) __builtin_nontemporal_store(val, reinterpret_cast<v4 *>(p + i * 4096));
    }
}

struct Allocation {
    uint64_t bytes = 0;                                // mapped (multiple of PIECE)
    std::vector<hipMemGenericAllocationHandle_t> h;    // pieces, in VA order
    uint32_t classes_found = 0, classes_used = 0;
    uint64_t groups_made = 0;
    double seconds = 0;
};

class Allocator {
  public:
    static Allocator &get() {
        static Allocator a;
        return a;
    }

    // Allocate `bytes` (>= MIN_BYTES) on the current device.  Returns
    // hipSuccess and *out, or an error (the caller then falls back).
    hipError_t alloc(uint64_t bytes, void **out) {
        std::lock_guard<std::mutex> lk(mu_);
        *out = nullptr;
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        const auto t0 = std::chrono::steady_clock::now();
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        const uint64_t npieces = (bytes + PIECE - 1) / PIECE;
        const uint64_t need_groups = (npieces + PIECES_PER_GROUP - 1) / PIECES_PER_GROUP;
        // a few more groups than needed, so that the choice can balance classes
        size_t fr = 0, tot = 0;
        uint64_t extra = need_groups / 2 + 2;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            const uint64_t headroom = 8 * GROUP, have = fr > headroom ? (fr - headroom) / GROUP : 0;
            if (have < need_groups) extra = 0;
            else extra = std::min(extra, have - need_groups);
        }
        const uint64_t ngroups = need_groups + extra;
        std::vector<hipMemGenericAllocationHandle_t> hs;
        hs.reserve(ngroups * PIECES_PER_GROUP);
        for (uint64_t i = 0; i < ngroups * PIECES_PER_GROUP; ++i) {
            hipMemGenericAllocationHandle_t h;
            e = hipMemCreate(&h, PIECE, &prop, 0);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                // out of memory for the extra groups: keep what we have if it is enough
                if (i >= npieces) break;
                for (auto x : hs) (void)hipMemRelease(x);
                return e;
            }
            hs.push_back(h);
        }
        const uint64_t have_groups = hs.size() / PIECES_PER_GROUP;
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;

        // ---- scratch mapping (creation order) and classification ----
        uint8_t *scratch = take_va(hs.size() * PIECE);
        std::vector<int> cls(have_groups, 0);
        uint32_t nclasses = 1;
        bool mapped = scratch != nullptr;
        size_t nmapped = 0;
        if (mapped) {
            for (; nmapped < hs.size(); ++nmapped)
                if (hipMemMap(scratch + nmapped * PIECE, PIECE, 0, hs[nmapped], 0) != hipSuccess) break;
            mapped = nmapped == hs.size() && hipMemSetAccess(scratch, hs.size() * PIECE, &acc, 1) == hipSuccess;
        }
        if (mapped && have_groups > 1) nclasses = classify(scratch, have_groups, cls);
        (void)hipGetLastError();
        for (size_t i = 0; i < nmapped; ++i) (void)hipMemUnmap(scratch + i * PIECE, PIECE);

        // ---- choose groups round-robin over the classes (largest first) ----
        std::vector<std::vector<uint64_t>> by(nclasses);
        for (uint64_t g = 0; g < have_groups; ++g) by[cls[g]].push_back(g);
        std::vector<int> order(nclasses);
        for (uint32_t c = 0; c < nclasses; ++c) order[c] = (int)c;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return by[a].size() > by[b].size(); });
        std::vector<uint64_t> chosen;
        std::vector<size_t> pos(nclasses, 0);
        std::vector<bool> used(nclasses, false);
        while (chosen.size() < need_groups) {
            bool any = false;
            for (int c : order) {
                if (chosen.size() == need_groups) break;
                if (pos[c] < by[c].size()) {
                    chosen.push_back(by[c][pos[c]++]);
                    used[c] = true;
                    any = true;
                }
            }
            if (!any) break;
        }
        std::vector<hipMemGenericAllocationHandle_t> pieces;
        for (uint64_t g : chosen)
            for (uint64_t i = 0; i < PIECES_PER_GROUP && pieces.size() < npieces; ++i)
                pieces.push_back(hs[g * PIECES_PER_GROUP + i]);
        {  // release every piece not used
            // the last chosen group may be partly used
            std::vector<bool> in_use(hs.size(), false);
            size_t k = 0;
            for (uint64_t g : chosen)
                for (uint64_t i = 0; i < PIECES_PER_GROUP && k < npieces; ++i, ++k) in_use[g * PIECES_PER_GROUP + i] = true;
            for (size_t i = 0; i < hs.size(); ++i)
                if (!in_use[i]) (void)hipMemRelease(hs[i]);
        }
        if (pieces.size() < npieces) {  // cannot happen unless creation failed midway
            for (auto x : pieces) (void)hipMemRelease(x);
            return hipErrorOutOfMemory;
        }

        // ---- final mapping: shuffled pieces behind a fresh VA range ----
        std::shuffle(pieces.begin(), pieces.end(), std::mt19937_64(0xCA4B0AD0u + npieces));
        uint8_t *va = take_va(npieces * PIECE);
        if (!va) {
            for (auto x : pieces) (void)hipMemRelease(x);
            return hipErrorOutOfMemory;
        }
        for (size_t i = 0; i < pieces.size(); ++i) {
            e = hipMemMap(va + i * PIECE, PIECE, 0, pieces[i], 0);
            if (e != hipSuccess) {
                for (size_t j = 0; j < i; ++j) (void)hipMemUnmap(va + j * PIECE, PIECE);
                for (auto x : pieces) (void)hipMemRelease(x);
                return e;
            }
        }
        e = hipMemSetAccess(va, npieces * PIECE, &acc, 1);
        if (e != hipSuccess) {
            for (size_t j = 0; j < pieces.size(); ++j) (void)hipMemUnmap(va + j * PIECE, PIECE);
            for (auto x : pieces) (void)hipMemRelease(x);
            return e;
        }
        Allocation A;
        A.bytes = npieces * PIECE;
        A.h = std::move(pieces);
        A.classes_found = nclasses;
        for (bool u : used) A.classes_used += u;
        A.groups_made = have_groups;
        A.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        live_[va] = std::move(A);
        *out = va;
        return hipSuccess;
    }

    // true if p came from alloc(); unmaps and releases it (its VA is retired).
    // Like hipFree it first waits for the device (work in flight may still
    // use the buffer), but outside the allocator's mutex: other threads'
    // allocations and frees are not held up behind that wait.
    bool free(void *p) {
        Allocation A;
        uint8_t *va = static_cast<uint8_t *>(p);
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = live_.find(va);
            if (it == live_.end()) return false;
            A = std::move(it->second);
            live_.erase(it);
        }
        (void)hipDeviceSynchronize();
        for (size_t i = 0; i < A.h.size(); ++i) (void)hipMemUnmap(va + i * PIECE, PIECE);
        for (auto x : A.h) (void)hipMemRelease(x);
        return true;
    }

    bool info(const void *p, Allocation *out) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = live_.find(static_cast<uint8_t *>(const_cast<void *>(p)));
        if (it == live_.end()) return false;
        out->bytes = it->second.bytes;
        out->classes_found = it->second.classes_found;
        out->classes_used = it->second.classes_used;
        out->groups_made = it->second.groups_made;
        out->seconds = it->second.seconds;
        return true;
    }

    // A never-used VA range of `bytes` (GROUP aligned) with nothing mapped:
    // the home of a Growable buffer.
    uint8_t *reserve(uint64_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        return take_va(bytes);
    }

  private:
    std::mutex mu_;
    std::map<uint8_t *, Allocation> live_;
    uint8_t *arena_ = nullptr;
    uint64_t arena_size_ = 0, arena_used_ = 0;

    // a never-used VA range of `bytes` (GROUP aligned)
    uint8_t *take_va(uint64_t bytes) {
        const uint64_t sz = (bytes + GROUP - 1) / GROUP * GROUP;
        if (!arena_ || arena_used_ + sz > arena_size_) {
            for (uint64_t want = 4ull << 40; want >= sz; want /= 2) {
                void *p = nullptr;
                if (hipMemAddressReserve(&p, want, GROUP, nullptr, 0) == hipSuccess && p) {
                    arena_ = static_cast<uint8_t *>(p);
                    arena_size_ = want;
                    arena_used_ = 0;
                    break;
                }
                (void)hipGetLastError();
                if (want == sz) return nullptr;
            }
            if (!arena_ || arena_used_ + sz > arena_size_) return nullptr;
        }
        uint8_t *r = arena_ + arena_used_;
        arena_used_ += sz;
        return r;
    }

    // Classes of `ng` groups mapped contiguously at `base`: greedy, one
    // representative group per class; returns the class count.
    uint32_t classify(uint8_t *base, uint64_t ng, std::vector<int> &cls) {
        hipStream_t s = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        auto rate = [&](uint64_t a, uint64_t b) {
            float best = 1e30f;
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0, s);
                hipLaunchKernelGGL(pair_write_kernel, dim3(512), dim3(256), 0, s, base + a * GROUP, base + b * GROUP, GROUP);
                (void)hipEventRecord(e1, s);
                float t = 0;
                if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess) return 0.0;
                best = std::min(best, t);
            }
            return 2.0 * GROUP / (best * 1e-3);
        };
        std::vector<uint64_t> reps;
        std::vector<double> self;
        for (uint64_t g = 0; g < ng; ++g) {
            cls[g] = -1;
            for (size_t r = 0; r < reps.size() && cls[g] < 0; ++r)
                if (rate(reps[r], g) < 1.12 * self[r]) cls[g] = (int)r;
            if (cls[g] < 0) {
                if ((int)reps.size() == MAX_CLASSES) { cls[g] = MAX_CLASSES - 1; continue; }
                cls[g] = (int)reps.size();
                reps.push_back(g);
                self.push_back(rate(g, g));
            }
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(s);
        return reps.empty() ? 1u : (uint32_t)reps.size();
    }
};

// A device buffer that grows in place: a large never-used VA range (from the
// allocator's arena, so never mapped twice) with physical pieces mapped
// behind it as it grows.  Growing copies nothing and waits for nothing (a
// hipMalloc + copy + hipFree growth synchronises the device each time); the
// bytes already written stay where they are, so work in flight over them is
// undisturbed.  Pieces double (8 MiB ... 1 GiB), so 1 GiB takes 8 maps.
// `grow` past the reserved range fails: the caller falls back (BaoHasher:
// one copy into plain memory).
struct Growable {
    uint8_t *va = nullptr;
    uint64_t va_bytes = 0, mapped = 0;
    std::vector<std::pair<hipMemGenericAllocationHandle_t, uint64_t>> h;  // piece, its size, in VA order

    // `reserve`: the VA range to take on the first call (GROUP multiples)
    hipError_t grow(uint64_t need, uint64_t reserve = 16 * GROUP) {
        if (need <= mapped) return hipSuccess;
        if (!va) {
            va_bytes = std::max<uint64_t>(reserve, (need + GROUP - 1) / GROUP * GROUP);
            va = Allocator::get().reserve(va_bytes);
            if (!va) return hipErrorOutOfMemory;
        }
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        while (mapped < need) {
            uint64_t sz = std::min<uint64_t>(GROUP, std::max<uint64_t>(PIECE, mapped));
            while (mapped + sz < need && sz < GROUP) sz *= 2;  // one map for a large append
            if (mapped + sz > va_bytes) return hipErrorOutOfMemory;
            hipMemGenericAllocationHandle_t x;
            if ((e = hipMemCreate(&x, sz, &prop, 0)) != hipSuccess) return e;
            if ((e = hipMemMap(va + mapped, sz, 0, x, 0)) != hipSuccess) {
                (void)hipMemRelease(x);
                return e;
            }
            if ((e = hipMemSetAccess(va + mapped, sz, &acc, 1)) != hipSuccess) {
                (void)hipMemUnmap(va + mapped, sz);
                (void)hipMemRelease(x);
                return e;
            }
            h.emplace_back(x, sz);
            mapped += sz;
        }
        return hipSuccess;
    }

    // Unmap and release every piece (the caller has synchronised the work
    // that used them); the VA range is retired with them.
    void release() {
        uint64_t off = 0;
        for (auto &x : h) {
            (void)hipMemUnmap(va + off, x.second);
            (void)hipMemRelease(x.first);
            off += x.second;
        }
        h.clear();
        va = nullptr;
        va_bytes = mapped = 0;
    }
};

}  // namespace hbm
}  // namespace chip
