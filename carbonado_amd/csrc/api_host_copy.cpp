// api_host_copy.cpp — host <-> HBM copies of the single-object calls: the
// pinned staging ring, the copy threads, NUMA placement of both, and
// chip_host_topology (where they sit).  Shared declarations: api_common.hpp.
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <condition_variable>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>

#include "api_common.hpp"

namespace chip {
namespace api {

// ---- host topology (NUMA) ------------------------------------------------------
// A GPU box is two sockets (NUMA nodes); each GPU hangs off one of them.  The
// pinned staging ring is read by the GPU's DMA engine and written by the copy
// threads, so both belong on the GPU's node: a ring or a copier on the other
// socket crosses the socket link on every byte (the BaoHasher line swung
// 16-29 GiB/s between processes, r7i, with unpinned threads free to run on
// either socket).  CHIP_NUMA=0 keeps the runtime's defaults (A/B).
namespace topo {
hipError_t host_alloc_on(void **p, size_t bytes, int node, unsigned flags = hipHostMallocDefault);

bool numa_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_NUMA");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

std::string read_file(const std::string &path) {
    std::ifstream f(path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

std::vector<int> parse_cpulist(const std::string &txt) {  // "0-63,128-191"
    std::vector<int> out;
    std::stringstream ss(txt);
    std::string part;
    while (std::getline(ss, part, ',')) {
        if (part.empty() || !std::isdigit((unsigned char)part[0])) continue;
        const size_t dash = part.find('-');
        const int a = std::atoi(part.c_str());
        const int b = dash == std::string::npos ? a : std::atoi(part.c_str() + dash + 1);
        for (int c = a; c <= b; ++c) out.push_back(c);
    }
    return out;
}

// node of every CPU (-1 unknown), from /sys/devices/system/node/node*/cpulist
const std::vector<int> &cpu_nodes() {
    static const std::vector<int> t = [] {
        std::vector<int> m;
        for (int node = 0; node < 64; ++node) {
            const std::string l = read_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
            if (l.empty()) continue;
            for (int c : parse_cpulist(l)) {
                if (c >= (int)m.size()) m.resize(c + 1, -1);
                m[c] = node;
            }
        }
        return m;
    }();
    return t;
}

int cpu_node(int cpu) {
    const auto &m = cpu_nodes();
    return cpu >= 0 && cpu < (int)m.size() ? m[cpu] : -1;
}

struct Gpu {
    std::string pci;        // e.g. 0000:75:00.0
    int node = -1;          // NUMA node of its PCI root, -1 unknown
    std::vector<int> cpus;  // its node's CPUs this process may run on
};

// The device's PCI address, node and local CPUs (sysfs), once per device.
const Gpu &gpu(int dev) {
    static std::mutex mu;
    static std::map<int, Gpu> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    Gpu g;
    char bdf[64] = {0};
    if (dev >= 0 && hipDeviceGetPCIBusId(bdf, sizeof bdf, dev) == hipSuccess) {
        for (char *q = bdf; *q; ++q) *q = (char)std::tolower((unsigned char)*q);
        g.pci = bdf;
        const std::string base = "/sys/bus/pci/devices/" + g.pci + "/";
        const std::string nd = read_file(base + "numa_node");
        g.node = nd.empty() ? -1 : std::atoi(nd.c_str());
        std::vector<int> local = parse_cpulist(read_file(base + "local_cpulist"));
        cpu_set_t aff;
        CPU_ZERO(&aff);
        if (sched_getaffinity(0, sizeof aff, &aff) == 0)
            for (int c : local)
                if (c < CPU_SETSIZE && CPU_ISSET(c, &aff)) g.cpus.push_back(c);
    } else {
        (void)hipGetLastError();
    }
    return cache.emplace(dev, g).first->second;
}

// NUMA node of the page holding p (move_pages(2) with no target = query)
int page_node(const void *p) {
    if (!p) return -1;
    void *pg = reinterpret_cast<void *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095));
    int status = -1;
    if (syscall(SYS_move_pages, 0, 1UL, &pg, nullptr, &status, 0) != 0) return -1;
    return status;
}

// hipHostMalloc with the pages placed on `node` (MPOL_PREFERRED for the call,
// hipHostMallocNumaUser so the runtime follows it), the thread's policy restored
hipError_t host_alloc_on(void **p, size_t bytes, int node, unsigned flags) {
    if (node < 0 || node >= 64 || !numa_on()) return hipHostMalloc(p, bytes, flags);
    constexpr int MPOL_DEFAULT_ = 0, MPOL_PREFERRED_ = 1;
    int old_mode = MPOL_DEFAULT_;
    unsigned long old_mask[16] = {0};
    const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, 16 * 64UL, nullptr, 0UL) == 0;
    unsigned long mask = 1UL << node;
    const bool set = syscall(SYS_set_mempolicy, MPOL_PREFERRED_, &mask, 64UL + 1) == 0;
    hipError_t e = hipHostMalloc(p, bytes, set ? (flags | hipHostMallocNumaUser) : flags);
    if (set) {
        if (saved) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == MPOL_DEFAULT_ ? nullptr : old_mask, 16 * 64UL);
        else (void)syscall(SYS_set_mempolicy, MPOL_DEFAULT_, nullptr, 0UL);
    }
    return e;
}

}  // namespace topo

// ---- host <-> HBM copies of the single-object calls -----------------------
// The runtime copies PAGEABLE host memory by pinning the caller's range: fast
// (55 GB/s) once a range is pinned, but pinning a range it has not seen costs
// ~24 ms per 34 MiB, and every fresh Vec / bytes the crate hands over is such a
// range.  Pageable buffers therefore go through a pinned 4 x 4 MiB ring, the
// CPU copy of one piece overlapping the DMA of the next (~1.4 ms per 34 MiB
// resident, ~6.4 ms into untouched memory, tools/pageable_probe.hip,
// profiles/r1w_pageable_probe.txt).  Small pageable copies take the ring
// too: direct, each costs ~22 us of API time whatever its size (r4c).
// Pinned (hipHostMalloc'd / registered) memory goes direct.
// CHIP_HOST_COPY=direct|staged forces one path (A/B runs).

int host_copy_mode() {  // 0 auto, 1 direct, 2 staged
    static const int m = [] {
        const char *e = std::getenv("CHIP_HOST_COPY");
        if (!e) return 0;
        if (!std::strcmp(e, "direct")) return 1;
        if (!std::strcmp(e, "staged")) return 2;
        return 0;
    }();
    return m;
}

bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error for the caller
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

bool staged(const void *host, size_t n) {
    const int m = host_copy_mode();
    if (m == 1 || !n) return false;
    return m == 2 || !host_pinned(host);
}

// Copies INTO the pinned ring go through host::ring_copy (non-temporal
// stores, host_stages.cpp); the other direction is a plain memcpy.
void copy_bytes(void *dst, const void *src, size_t n, bool nt) {
    if (nt) host::ring_copy(dst, src, n);
    else std::memcpy(dst, src, n);
}

// memcpy between the ring and pageable memory on a few threads: one thread
// moves ~20 GB/s, the ring DMA 55 GB/s.  A persistent pool (CHIP_COPY_THREADS
// total, default 8, 1 = the calling thread only; 8 over 4: host scrub() +15 %,
// 16 MiB encode() -14 %, r5a: the copies into fresh pages are page-fault bound); a caller that finds the
// pool busy (another thread's copy) copies alone.
class CopyPool {
  public:
    static CopyPool &get() {
        static CopyPool *p = new CopyPool();  // never destroyed: workers park on the condvar at exit
        return *p;
    }
    // nt: dst is the pinned ring, read next by the DMA engine (copy_bytes)
    void copy(void *dst, const void *src, size_t n, bool nt = false) {
        // (a forked child has no workers: it copies alone)
        if (workers_ == 0 || n < (size_t(1) << 20) || getpid() != pid_ || !job_.try_lock()) {
            copy_bytes(dst, src, n, nt);
            return;
        }
        const size_t parts = workers_ + 1;
        size_t part = (n + parts - 1) / parts;
        part = (part + 65535) & ~size_t(65535);
        {
            std::lock_guard<std::mutex> lk(mu_);
            d_ = static_cast<uint8_t *>(dst);
            s_ = static_cast<const uint8_t *>(src);
            n_ = n;
            part_ = part;
            nt_ = nt;
            pending_ = workers_;
            ++gen_;
        }
        cv_.notify_all();
        copy_bytes(dst, src, std::min(part, n), nt);
        {
            std::unique_lock<std::mutex> lk(mu_);
            done_.wait(lk, [&] { return pending_ == 0; });
        }
        job_.unlock();
    }

    int workers() const { return workers_; }
    bool pinned() const { return pinned_; }
    int node() const { return node_; }
    // CPU each worker last copied on (-1: no job yet)
    std::vector<int> last_cpus() const {
        std::vector<int> v;
        for (int i = 1; i <= workers_ && i < MAXW; ++i) v.push_back(last_cpu_[i].load());
        return v;
    }

  private:
    static constexpr int MAXW = 33;
    CopyPool() {
        int t = 8;
        if (const char *e = std::getenv("CHIP_COPY_THREADS")) t = std::max(1, std::min(32, std::atoi(e)));
        workers_ = t - 1;
        pid_ = getpid();
        // workers on the GPU's node, next to the ring they fill (topo::)
        const int dev = g_device;
        if (topo::numa_on() && dev >= 0) {
            const topo::Gpu &g = topo::gpu(dev);
            if (!g.cpus.empty()) {
                CPU_ZERO(&cpus_);
                for (int c : g.cpus) CPU_SET(c, &cpus_);
                pinned_ = true;
                node_ = g.node;
            }
        }
        for (int i = 0; i < MAXW; ++i) last_cpu_[i] = -1;
        for (int i = 1; i <= workers_; ++i) std::thread([this, i] { run(i); }).detach();
    }
    void run(int i) {
        if (pinned_) (void)pthread_setaffinity_np(pthread_self(), sizeof cpus_, &cpus_);
        uint64_t seen = 0;
        for (;;) {
            uint8_t *d;
            const uint8_t *s;
            size_t n, part;
            bool nt;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                d = d_, s = s_, n = n_, part = part_, nt = nt_;
            }
            const size_t lo = std::min(n, i * part), hi = std::min(n, lo + part);
            if (hi > lo) copy_bytes(d + lo, s + lo, hi - lo, nt);
            if (i < MAXW) last_cpu_[i] = sched_getcpu();
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int workers_ = 0;
    bool pinned_ = false;
    int node_ = -1;
    cpu_set_t cpus_;
    std::atomic<int> last_cpu_[MAXW];
    pid_t pid_ = 0;
    std::mutex job_, mu_;
    std::condition_variable cv_, done_;
    uint64_t gen_ = 0;
    int pending_ = 0;
    uint8_t *d_ = nullptr;
    const uint8_t *s_ = nullptr;
    size_t n_ = 0, part_ = 0;
    bool nt_ = false;
};

hipError_t grow_pinned_local(DevBuf &b, size_t bytes, unsigned flags) {
    if (bytes == 0) bytes = 16;
    if (b.cap >= bytes) return hipSuccess;
    if (b.p) {
        hipError_t e = hipHostFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.cap = 0;
    }
    const size_t cap = ((bytes + (bytes >> 3)) + 4095) & ~size_t(4095);
    const int dev = g_device;
    hipError_t e = topo::host_alloc_on(&b.p, cap, dev >= 0 ? topo::gpu(dev).node : -1, flags);
    if (e != hipSuccess) {
        b.p = nullptr;
        return e;
    }
    b.cap = cap;
    return hipSuccess;
}


hipError_t stage_slot(Staging &sg, int k) {  // wait until ring slot k is free
    if (!sg.armed[k]) return hipSuccess;
    sg.armed[k] = false;
    return hipEventSynchronize(sg.ev[k]);
}

hipError_t stage_init(Staging &sg) {
    if (sg.ring) return hipSuccess;
    const int dev = g_device;
    hipError_t e = topo::host_alloc_on(reinterpret_cast<void **>(&sg.ring), Staging::R * Staging::PIECE,
                                       dev >= 0 ? topo::gpu(dev).node : -1);
    if (e != hipSuccess) {
        sg.ring = nullptr;
        return e;
    }
    for (int k = 0; k < Staging::R && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&sg.ev[k], hipEventDisableTiming);
    return e;
}

// Enqueue host -> HBM on s.  On return `src` may be reused (its bytes are in
// the ring or already copied); later work on s sees the data.
hipError_t h2d(Staging &sg, void *dst, const void *src, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (!staged(src, n)) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    hipError_t e = stage_init(sg);
    for (size_t off = 0; off < n && e == hipSuccess; off += Staging::PIECE) {
        const size_t len = std::min(Staging::PIECE, n - off);
        const int k = sg.next++ % Staging::R;
        if ((e = stage_slot(sg, k)) != hipSuccess) break;
        CopyPool::get().copy(sg.ring + k * Staging::PIECE, static_cast<const uint8_t *>(src) + off, len, true);
        e = hipMemcpyAsync(static_cast<uint8_t *>(dst) + off, sg.ring + k * Staging::PIECE, len,
                           hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(sg.ev[k], s);
        if (e == hipSuccess) sg.armed[k] = true;
    }
    return e;
}

// The caller's output buffer, about to be written by the host threads: a
// fresh allocation (a Rust Vec::with_capacity per call) takes a page fault per
// 4 KiB on first touch, ~7 ms for a 35 MB level-12 stream of a 16 MiB object
// (r11k).  Its 2 MiB-aligned interior is advised onto transparent huge pages
// (advice only: no effect on pages already present, none on the bytes; a
// failure is ignored).  CHIP_OUT_THP=0 turns it off.
void advise_huge(void *p, uint64_t n) {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_OUT_THP");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    constexpr uintptr_t H = uintptr_t(2) << 20;
    if (!on || n < 2 * H) return;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + H - 1) & ~(H - 1);
    const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + n) & ~(H - 1);
    if (b > a) (void)madvise(reinterpret_cast<void *>(a), b - a, MADV_HUGEPAGE);
}

// HBM -> host after the work already on s, in two halves so the caller can
// work between them: d2h_begin enqueues the first ring pieces' DMA, d2h_end
// copies every piece out (enqueuing the rest as ring slots free up) and
// returns when `dst` holds the bytes.
hipError_t d2h_begin(Staging &sg, D2h &t, void *dst, const void *src, size_t n, hipStream_t s) {
    t = D2h{dst, src, n, s, 0, 0, false};
    if (!n) return hipSuccess;
    if (!staged(dst, n)) {
        t.direct = true;
        return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s);
    }
    hipError_t e = stage_init(sg);
    if (e != hipSuccess) return e;
    advise_huge(dst, n);  // the copy threads fault its pages in next
    t.np = (n + Staging::PIECE - 1) / Staging::PIECE;
    t.base = sg.next;
    sg.next += (unsigned)t.np;
    for (size_t j = 0; j < t.np && j < (size_t)Staging::R && e == hipSuccess; ++j) e = d2h_issue(sg, t, j);
    return e;
}

hipError_t d2h_issue(Staging &sg, const D2h &t, size_t j) {
    const int k = (int)((t.base + j) % Staging::R);
    hipError_t r = stage_slot(sg, k);
    const size_t off = j * Staging::PIECE;
    if (r == hipSuccess)
        r = hipMemcpyAsync(sg.ring + k * Staging::PIECE, static_cast<const uint8_t *>(t.src) + off,
                           std::min(Staging::PIECE, t.n - off), hipMemcpyDeviceToHost, t.s);
    if (r == hipSuccess) r = hipEventRecord(sg.ev[k], t.s);
    if (r == hipSuccess) sg.armed[k] = true;
    return r;
}

hipError_t d2h_end(Staging &sg, const D2h &t) {
    if (!t.n) return hipSuccess;
    if (t.direct) return hipStreamSynchronize(t.s);
    hipError_t e = hipSuccess;
    for (size_t j = 0; j < t.np && e == hipSuccess; ++j) {
        const int k = (int)((t.base + j) % Staging::R);
        if ((e = stage_slot(sg, k)) != hipSuccess) break;
        const size_t off = j * Staging::PIECE;
        CopyPool::get().copy(static_cast<uint8_t *>(t.dst) + off, sg.ring + k * Staging::PIECE,
                             std::min(Staging::PIECE, t.n - off));
        if (j + Staging::R < t.np) e = d2h_issue(sg, t, j + Staging::R);
    }
    return e;
}

hipError_t d2h(Staging &sg, void *dst, const void *src, size_t n, hipStream_t s) {
    D2h t;
    hipError_t e = d2h_begin(sg, t, dst, src, n, s);
    return e == hipSuccess ? d2h_end(sg, t) : e;
}

}  // namespace api
}  // namespace chip

using namespace chip;
using namespace chip::api;

extern "C" {

int chip_host_topology(char *out, uint64_t cap, uint64_t *len) {
    if (!len) return CHIP_ERR_INVALID_ARG;
    Ctx *c = nullptr;
    int st = ctx_get(&c);
    if (st != CHIP_OK) return st;
    const topo::Gpu &g = topo::gpu(c->dev);
    CopyPool &pool = CopyPool::get();
    std::map<int, int> by_node;  // copy workers by the node of the CPU they last ran a copy on
    for (int cpu : pool.last_cpus()) ++by_node[cpu < 0 ? -2 : topo::cpu_node(cpu)];
    cpu_set_t aff;
    CPU_ZERO(&aff);
    const int naff = sched_getaffinity(0, sizeof aff, &aff) == 0 ? CPU_COUNT(&aff) : -1;
    const int here = sched_getcpu();
    std::string j = "{\"numa_placement\": " + std::string(topo::numa_on() ? "true" : "false") +
                    ", \"gpu_pci\": \"" + g.pci + "\", \"gpu_node\": " + std::to_string(g.node) +
                    ", \"gpu_local_cpus_allowed\": " + std::to_string(g.cpus.size()) +
                    ", \"process_cpus_allowed\": " + std::to_string(naff) +
                    ", \"caller_cpu_node\": " + std::to_string(here < 0 ? -1 : topo::cpu_node(here)) +
                    ", \"ring_node\": " + std::to_string(c->stage.ring ? topo::page_node(c->stage.ring) : -1) +
                    ", \"copy_workers\": " + std::to_string(pool.workers()) +
                    ", \"copy_workers_pinned\": " + std::string(pool.pinned() ? "true" : "false") +
                    ", \"copy_workers_by_last_cpu_node\": {";
    bool first = true;
    for (auto &kv : by_node) {
        j += (first ? "\"" : ", \"") + (kv.first == -2 ? std::string("idle") : std::to_string(kv.first)) + "\": " +
             std::to_string(kv.second);
        first = false;
    }
    j += "}}";
    *len = j.size() + 1;
    if (!out || cap < *len) return CHIP_ERR_BUFFER_TOO_SMALL;
    std::memcpy(out, j.c_str(), j.size() + 1);
    return CHIP_OK;
}

// torch.cuda.memory.CUDAPluggableAllocator hooks over chip_device_alloc/free
void *chip_torch_alloc(ssize_t size, int device, void *stream) {
    (void)stream;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    void *p = nullptr;
    return chip_device_alloc(size > 0 ? (uint64_t)size : 0, &p) == CHIP_OK ? p : nullptr;
}

}  // extern "C"
