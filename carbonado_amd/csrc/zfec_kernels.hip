// zfec_kernels.hip — K1/K2: GF(2^8) stripe matrix-apply for gfx950.
//
// Replaces the arithmetic of zfec-rs 0.1.0's Fec::encode / Fec::decode
// (called at /root/reference/src/encoding.rs:61-62 and decoding.rs:28-29).
// Encode: parity S_i[t] = XOR_j E[i][j] * D_j[t] for k <= i < m, with the
// k data shards D_j = contiguous C-byte slices of the zero-padded input
// (encoding.rs:53-55); the output is shard-major [S0|..|S(m-1)] (encoding.rs:70-78).
// Decode with erasures is the same apply with rows of the inverted share matrix.
//
// Design (HBM-bound byte streaming; no MFMA: GF(2^8) products are table work):
//  * One lane owns 16 byte-columns of every input shard: k coalesced
//    global_load_dwordx4 per tile, m global_store_dwordx4 (nontemporal) per tile.
//  * Packed-coefficient table in LDS: entry T_s[x] holds the products of byte x
//    with shard s's coefficient in each computed row, packed 4 rows per dword
//    (NG dwords).  One ds_read per input byte yields 4*NG parity contributions;
//    a 4x4 byte transpose (v_perm_b32) turns column-packed sums into row streams.
//  * Bank-conflict-free lookups: the table is replicated R = 32/K times; lane
//    group G = (lane&31)/R walks the shards in the rotated order (j+G) mod K, so
//    the 32 lanes of an LDS lane-group read 32 distinct banks for any data.
//  * Persistent grid (occupancy x CUs), grid-stride over (object, 4 KiB column
//    tile).  No inter-workgroup communication, no atomics.
#include "chip_internal.hpp"
#include "gf256.hpp"
#include "zfec_device.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

namespace chip {

namespace {

using namespace zf;

// ---- generic fallback: any k (<= 256) and any number of output rows ----
// One thread = 16 columns of one output row; full 64 KiB GF multiplication
// table in LDS.  Used only outside the fast kernel's (K <= 16, rows <= 8) range.
struct GenericArgs {
    const uint8_t *in;
    uint8_t *out;
    uint64_t in_stride, out_stride, valid, C, count;
    uint32_t k, rows;
    const uint64_t *in_off;   // [k]
    const uint64_t *out_off;  // [rows]
    const uint8_t *coef;      // [rows][k]
    const uint8_t *multab;    // [256][256]
};

__global__ __launch_bounds__(TPB) void gf_apply_generic_kernel(GenericArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt[];
    for (int i = threadIdx.x; i < 65536 / 16; i += TPB)
        reinterpret_cast<u32x4 *>(mt)[i] = reinterpret_cast<const u32x4 *>(a.multab)[i];
    __syncthreads();
    const uint64_t cols = (a.C + VEC - 1) / VEC;
    const uint64_t total = a.count * a.rows * cols;
    for (uint64_t w = (uint64_t)blockIdx.x * TPB + threadIdx.x; w < total;
         w += (uint64_t)gridDim.x * TPB) {
        const uint64_t cidx = w % cols;
        const uint64_t rr = (w / cols) % a.rows;
        const uint64_t obj = w / cols / a.rows;
        const uint64_t col = cidx * VEC;
        const uint8_t *ib = a.in + obj * a.in_stride;
        uint32_t acc[4] = {0u, 0u, 0u, 0u};
        for (uint32_t j = 0; j < a.k; ++j) {
            const uint8_t c = a.coef[rr * a.k + j];
            if (!c) continue;
            const u32x4 x = load16_masked(ib, a.in_off[j] + col, a.valid);
            const uint8_t *row = mt + c * 256;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const uint32_t xd = comp(x, d);
                acc[d] ^= (uint32_t)row[xd & 0xFF] | (uint32_t)row[(xd >> 8) & 0xFF] << 8 |
                          (uint32_t)row[(xd >> 16) & 0xFF] << 16 | (uint32_t)row[xd >> 24] << 24;
            }
        }
        u32x4 o = {acc[0], acc[1], acc[2], acc[3]};
        *reinterpret_cast<u32x4 *>(a.out + obj * a.out_stride + a.out_off[rr] + col) = o;
    }
}

// ---- box ceiling: gf_apply's memory pattern without the arithmetic ----------
// The same loads (K masked 16-B loads per lane per column tile, shards walked
// in the lane group's rotated order, super-tiles of U tiles with the next
// one's loads in flight), the same stores (K copies + NP computed rows, 16 B
// per lane each, NT as the product), the same run queue, grid and LDS
// footprint (set by the launch), but computed row q is the XOR of the K
// loads and the byte q instead of K*16 table lookups.  What this box's HBM gives the
// headline's access pattern on the caller's buffers: bench.py prices the
// headline against it (frac_of_box_ceiling) so a slow box explains itself.
template <int K, int NP, int U, bool NT>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(2))) void hbm_pattern_kernel(ApplyArgs a) {
    constexpr int R = replicas_for(K);
    const int grp = ((int)threadIdx.x & 31) / R;
    uint64_t ioff[K], coff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        ioff[j] = a.in_off[(j + grp) % K];
        coff[j] = a.copy_off[(j + grp) % K];
    }
    const uint64_t spo = (a.tiles_per_obj + U - 1) / U;
    __shared__ uint32_t q_slot[2];
    QueueIter<6> iter(spo * a.count, a.chunk, a.queue, q_slot, a.xcd_mask);
    auto load_tile = [&](uint64_t t, u32x4 (&v)[U][K]) {
        const uint64_t obj = t / spo;
        const uint64_t col0 = (t - obj * spo) * (uint64_t)(U * TILE) + threadIdx.x * VEC;
        const uint8_t *ib = a.in + obj * a.in_stride;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint64_t col = col0 + (uint64_t)u * TILE;
                v[u][j] = col < a.C ? load16_masked(ib, ioff[j] + col, a.valid) : u32x4{0u, 0u, 0u, 0u};
            }
    };
    uint64_t st;
    bool have = iter.next(st);
    u32x4 v[U][K];
    if (have) load_tile(st, v);
    while (have) {
        uint64_t st_next;
        const bool have_next = iter.next(st_next);
        u32x4 vn[U][K];
        if (have_next) load_tile(st_next, vn);
        const uint64_t obj = st / spo;
        const uint64_t col0 = (st - obj * spo) * (uint64_t)(U * TILE) + threadIdx.x * VEC;
        uint8_t *ob = a.out + obj * a.out_stride;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t col = col0 + (uint64_t)u * TILE;
            if (col >= a.C) continue;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (coff[j] != NO_OUT) store16<NT>(ob + coff[j] + col, v[u][j]);
            u32x4 x = v[u][0];  // the XOR of all K shards: the same whatever the lane's shard order
#pragma unroll
            for (int j = 1; j < K; ++j) x ^= v[u][j];
#pragma unroll
            for (int q = 0; q < NP; ++q)
                if (a.par_off[q] != NO_OUT) store16<NT>(ob + a.par_off[q] + col, x ^ (0x01010101u * (uint32_t)q));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) v[u][j] = vn[u][j];
        st = st_next;
        have = have_next;
    }
    iter.finish();
}

// ---- host side ----------------------------------------------------------
typedef void (*KernelFn)(ApplyArgs);

// Schedule.  Every shape walks its column tiles through the
// dynamic per-XCD run queue (MAP 6, QueueIter): runs of ZF_CHUNK tiles (256
// KiB per shard) dealt from 8 contiguous shares of the batch, one per XCD,
// and once an XCD's share is done it takes runs of the others'.  The XCDs
// do not stream at the same rate (odd XCDs ~20 % slower on every box
// measured, tools/zfec_timeline), so the static XCD-grouped order this
// replaces (MAP 3) ended with half the chip idle for the last ~1 ms of a
// 10 ms launch; the queue ends every XCD within ~0.1 ms (+2.5-3 % on the
// headline, and it needs no per-box schedule choice).
constexpr int ZF_MAP = 6;
constexpr bool ZF_NT = true;
constexpr uint64_t ZF_CHUNK = 64;   // tiles per run (U = 1 tiles; U = 2 super-tiles run ZF_CHUNK / 2)
constexpr uint64_t ZF_BL_RUN = 32;  // bao-layout kernel: consecutive 1 KiB units per wave run

// Wide stripes (K > 4): pin the XOR partial sums every shard (SB = 1) so the
// K*16 table lookups are not all live at once — without it K = 8 compiles to
// 256 VGPR + 90 AGPR, one wave per SIMD — and prefetch the next tile's shards
// into registers (K <= 8; K = 16 has no registers to spare).  8 computed
// rows (NG = 2): plain stores measured +1-3% over nontemporal at 2
// workgroups/CU (tools/zfec_tune, 8-of-16 sweep in DESIGN.md).
// The 4-of-8 shape (K = 4, NG = 1): super-tiles of 2 column tiles, the next
// one's shards prefetched into registers, 2 workgroups/CU (160 VGPRs).
struct KernelInfo {
    KernelFn fn;
    size_t lds;
    int u;        // column tiles per super-tile (the kernel's U)
    int bpc_cap;  // workgroups per CU to launch (0 = occupancy limit)
};

#ifndef ZF_NTL_DEF
#define ZF_NTL_DEF 0
#endif
template <int K, int NG>
struct ApplyCfg {
    static constexpr bool K4 = K == 4 && NG == 1;  // the 4-of-8 shape
    static constexpr int U = K4 ? 2 : 1;
    static constexpr int WPE = (K > 4 || K4) ? 2 : 1;
    static constexpr int SB = K > 4 ? 1 : 0;
    static constexpr bool PF = K > 4 ? K <= 8 : K4;
    static constexpr bool NT = K > 4 ? (NG == 1 && ZF_NT) : ZF_NT;
    static constexpr bool NTL = K4 && ZF_NTL_DEF;
    static constexpr int BPC_CAP = K4 ? 2 : 0;
};

// The product's zfec apply kernel for K input shards and NG dword groups of
// computed rows (4 NG rows), in its ApplyCfg configuration.
template <int K, int NG>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(ApplyCfg<K, NG>::WPE))) void zfec_apply_kernel(
    ApplyArgs a) {
    using C = ApplyCfg<K, NG>;
    gf_apply_body<K, NG, C::U, ZF_MAP, C::NT, 0, C::WPE, C::SB, C::PF, C::NTL>(a);
}

template <int K, int NG>
KernelInfo make_info() {
    constexpr int R = replicas_for(K);
    KernelInfo ki;
    ki.lds = (size_t)256 * K * R * 4 * NG;
    ki.fn = zfec_apply_kernel<K, NG>;
    ki.u = ApplyCfg<K, NG>::U;
    ki.bpc_cap = ApplyCfg<K, NG>::BPC_CAP;
    return ki;
}

bool lookup_fast(int k, int ng, KernelInfo &out) {
#define CHIP_CASE(KK)                                                        \
    case KK:                                                                 \
        out = (ng == 1) ? make_info<KK, 1>() : make_info<KK, 2>();           \
        return true;
    switch (k) {
        CHIP_CASE(1) CHIP_CASE(2) CHIP_CASE(3) CHIP_CASE(4) CHIP_CASE(5)
        CHIP_CASE(6) CHIP_CASE(7) CHIP_CASE(8) CHIP_CASE(16)
        default: return false;
    }
#undef CHIP_CASE
}

struct DevTable {
    void *ptr = nullptr;
    size_t bytes = 0;
};

std::mutex g_mu;
std::map<std::vector<uint8_t>, DevTable> g_tables;  // key: device, k, ng, coef bytes
std::map<std::pair<KernelFn, size_t>, int> g_grid;
std::map<int, uint8_t *> g_multab;                  // per device

// Run-queue counters (QueueIter) per stream: launches on one stream run one
// after another, and each launch leaves its counters zero (its last
// workgroup resets them), so a stream's launches can share one block.  Every
// stream gets a block of its own: a destroyed stream's block first, else a
// never-used one, and when a pool of QUEUE_SLOTS blocks is used up another
// pool is allocated.  No two live streams ever share a block (two persistent
// launches on one block lose or repeat tiles).  Streams the library does not
// own (torch's, a Rust caller's) keep their block for the process lifetime:
// 4 KiB per distinct stream.  Block layout (uint32 words): K1 0-256 (8
// counters 32 apart + the done counter), K13 QUEUE_K13 + {0, 32}, K3
// QUEUE_K3 + {0, 32}.  (The block was 2 KiB while K13 and K3 already used
// words 512-672, i.e. the NEXT stream's K1 counters: a K1 launch on one
// thread's stream beside a K13 / K3 launch on the neighbouring stream could
// lose or repeat column tiles.)
constexpr int QUEUE_SLOTS = 256;
constexpr size_t QUEUE_BYTES = 4096;
static_assert(QUEUE_K3 + 33 <= (int)(QUEUE_BYTES / 4) && QUEUE_K13 + 33 <= QUEUE_K3 && 257 <= QUEUE_K13,
              "run-queue block layout");
std::map<int, std::vector<uint8_t *>> g_queue_pools;        // per device: pools of QUEUE_SLOTS blocks
std::map<std::pair<int, hipStream_t>, uint32_t *> g_queue;  // (device, stream) -> counters
std::map<int, std::vector<uint32_t *>> g_queue_free;        // per device: blocks of destroyed streams
std::map<int, size_t> g_queue_next;                          // per device: next never-used block of the last pool

hipError_t queue_for(hipStream_t stream, uint32_t **out) {
    const int dev = selected_device();
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(dev, stream);
    auto it = g_queue.find(key);
    if (it != g_queue.end()) { *out = it->second; return hipSuccess; }
    uint32_t *q;
    std::vector<uint32_t *> &fl = g_queue_free[dev];
    if (!fl.empty()) {  // a destroyed stream's block (its launches left it zero)
        q = fl.back();
        fl.pop_back();
    } else {
        std::vector<uint8_t *> &pools = g_queue_pools[dev];
        size_t &nx = g_queue_next[dev];
        if (pools.empty() || nx == (size_t)QUEUE_SLOTS) {
            uint8_t *d = nullptr;
            hipError_t e = hipMalloc(&d, QUEUE_SLOTS * QUEUE_BYTES);
            if (e != hipSuccess) return e;
            // zeroed on a private stream and waited for, so the pool is zero
            // before any stream's launch reads it, whatever that stream's flags
            hipStream_t zs = nullptr;
            e = hipStreamCreateWithFlags(&zs, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipMemsetAsync(d, 0, QUEUE_SLOTS * QUEUE_BYTES, zs);
            if (e == hipSuccess) e = hipStreamSynchronize(zs);
            if (zs) (void)hipStreamDestroy(zs);
            if (e != hipSuccess) { (void)hipFree(d); return e; }
            pools.push_back(d);
            nx = 0;
        }
        q = reinterpret_cast<uint32_t *>(pools.back() + nx * QUEUE_BYTES);
        ++nx;
    }
    g_queue[key] = q;
    *out = q;
    return hipSuccess;
}

size_t queue_blocks_in_use() {
    const int dev = selected_device();
    std::lock_guard<std::mutex> lk(g_mu);
    size_t n = 0;
    for (const auto &kv : g_queue)
        if (kv.first.first == dev) ++n;
    return n;
}

int grid_for(const KernelInfo &ki) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(ki.fn, ki.lds);
    auto it = g_grid.find(key);
    if (it != g_grid.end()) return it->second;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(ki.fn),
                                                     TPB, ki.lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    if (ki.bpc_cap > 0 && per_cu > ki.bpc_cap) per_cu = ki.bpc_cap;
    if (const char *e = std::getenv("CHIP_ZF_GRID_BPC"))  // calibration override (tools)
        per_cu = std::max(1, std::atoi(e));
    const int g = per_cu * num_cus();
    g_grid[key] = g;
    return g;
}

// Packed table for the fast kernel: entry [s][x] = NG dwords, byte (4g+q) of
// dword g = coef[4g+q][s] * x.
hipError_t device_table(const GfPlan &p, int ng, const void **out) {
    std::vector<uint8_t> key;
    key.push_back((uint8_t)selected_device());  // device-side tables live on the process's device
    key.push_back((uint8_t)p.k);
    key.push_back((uint8_t)ng);
    key.insert(key.end(), p.coef.begin(), p.coef.end());
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_tables.find(key);
    if (it != g_tables.end()) { *out = it->second.ptr; return hipSuccess; }
    const Gf256 &gf = Gf256::get();
    std::vector<uint32_t> host((size_t)p.k * 256 * ng, 0u);
    for (uint32_t s = 0; s < p.k; ++s)
        for (int x = 0; x < 256; ++x)
            for (uint32_t row = 0; row < p.np; ++row) {
                const uint8_t prod = gf.mul(p.coef[row * p.k + s], (uint8_t)x);
                host[((size_t)s * 256 + x) * ng + row / 4] |= (uint32_t)prod << (8 * (row % 4));
            }
    DevTable t;
    t.bytes = host.size() * 4;
    hipError_t e = hipMalloc(&t.ptr, t.bytes);
    if (e != hipSuccess) return e;
    e = hipMemcpy(t.ptr, host.data(), t.bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(t.ptr); return e; }
    g_tables[key] = t;
    *out = t.ptr;
    return hipSuccess;
}

hipError_t multab_device(const uint8_t **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    uint8_t *&mt = g_multab[selected_device()];
    if (!mt) {
        const Gf256 &gf = Gf256::get();
        std::vector<uint8_t> h(65536);
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b) h[a * 256 + b] = gf.mul((uint8_t)a, (uint8_t)b);
        uint8_t *d = nullptr;
        hipError_t e = hipMalloc(&d, 65536);
        if (e != hipSuccess) return e;
        e = hipMemcpy(d, h.data(), 65536, hipMemcpyHostToDevice);
        if (e != hipSuccess) { (void)hipFree(d); return e; }
        mt = d;
    }
    *out = mt;
    return hipSuccess;
}

hipError_t apply_generic(const GfPlan &p, const GfLaunch &L, hipStream_t stream) {
    const uint8_t *mt = nullptr;
    hipError_t e = multab_device(&mt);
    if (e != hipSuccess) return e;
    const uint32_t rows = (uint32_t)p.g_out_off.size();
    // small per-launch descriptor block: in_off, out_off, coef
    const size_t b_in = p.k * 8, b_out = rows * 8, b_coef = (size_t)rows * p.k;
    std::vector<uint8_t> blob(b_in + b_out + b_coef);
    std::memcpy(blob.data(), p.g_in_off.data(), b_in);
    std::memcpy(blob.data() + b_in, p.g_out_off.data(), b_out);
    std::memcpy(blob.data() + b_in + b_out, p.g_coef.data(), b_coef);
    void *d = nullptr;
    e = hipMallocAsync(&d, blob.size(), stream);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(d, blob.data(), blob.size(), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    GenericArgs a;
    a.in = L.in; a.out = L.out; a.in_stride = L.in_stride; a.out_stride = L.out_stride;
    a.valid = L.valid; a.C = L.C; a.count = L.count; a.k = p.k; a.rows = rows;
    a.in_off = reinterpret_cast<const uint64_t *>(d);
    a.out_off = reinterpret_cast<const uint64_t *>(static_cast<uint8_t *>(d) + b_in);
    a.coef = static_cast<const uint8_t *>(d) + b_in + b_out;
    a.multab = mt;
    const uint64_t work = L.count * rows * ((L.C + VEC - 1) / VEC);
    uint64_t blocks = (work + TPB - 1) / TPB;
    const uint64_t cap = (uint64_t)num_cus() * 2;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(gf_apply_generic_kernel, dim3((unsigned)blocks), dim3(TPB), 65536, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the memcpy above captured `blob` synchronously into the stream order;
    // free the descriptor once the kernel has consumed it
    return hipFreeAsync(d, stream);
}

hipError_t gf_apply_pass(const GfPlan &p, const GfLaunch &L, hipStream_t stream,
                         uint32_t row0, uint32_t nrows, bool copies) {
    const int ng = nrows > 4 ? 2 : 1;
    KernelInfo ki;
    if (!lookup_fast((int)p.k, ng, ki)) return hipErrorInvalidValue;
    ApplyArgs a;
    std::memset(&a, 0, sizeof a);
    a.in = L.in; a.out = L.out;
    a.in_stride = L.in_stride; a.out_stride = L.out_stride;
    a.bao_off = L.bao_off;
    a.bao_n = L.bao_off ? (L.C / 1024) * (p.k + p.np) : 0;  // m*C/1024 chunks
    KernelFn fn = ki.fn;
    size_t lds = ki.lds;
    const bool bl = L.bao_off != nullptr;
    if (bl) {  // bao layout: the dedicated 4-of-8 kernel, one pass (copies + all 4 parity rows)
        if (p.k != 4 || p.np != 4 || L.C % 1024 || !copies || row0 != 0) return hipErrorInvalidValue;
        fn = gf_apply_bl_kernel<ZF_NT>;
        ki.fn = fn;  // occupancy of the kernel actually launched
        ki.u = 1;
        ki.bpc_cap = 0;
    }
    a.valid = L.valid; a.C = L.C;
    a.tiles_per_obj = (L.C + TILE - 1) / TILE;
    a.total_tiles = a.tiles_per_obj * L.count;
    a.count = L.count;
    for (int j = 0; j < ZF_MAXK; ++j) {
        a.in_off[j] = j < (int)p.k ? p.in_off[j] : 0;
        a.copy_off[j] = (copies && j < (int)p.k) ? p.copy_off[j] : NO_OUT;
    }
    for (uint32_t q = 0; q < (uint32_t)ZF_MAXP; ++q) a.par_off[q] = q < nrows ? p.comp_off[row0 + q] : NO_OUT;
    GfPlan sub;
    sub.k = p.k;
    sub.np = nrows;
    sub.coef.assign(p.coef.begin() + (size_t)row0 * p.k, p.coef.begin() + (size_t)(row0 + nrows) * p.k);
    hipError_t e = device_table(sub, ng, &a.table);
    if (e != hipSuccess) return e;
    if (!bl && (e = queue_for(stream, &a.queue)) != hipSuccess) return e;
    int grid_cap = grid_for(ki);
    if (L.wg_per_cu > 0 && grid_cap > L.wg_per_cu * num_cus()) grid_cap = L.wg_per_cu * num_cus();
    // the kernel walks super-tiles of ki.u column tiles (never across objects)
    const uint64_t units = ((a.tiles_per_obj + ki.u - 1) / ki.u) * L.count;
    uint64_t grid = units < (uint64_t)grid_cap ? units : (uint64_t)grid_cap;
    if (grid >= 8) grid = grid / 8 * 8;  // XCD grouping needs a multiple of 8
    // runs of up to ZF_CHUNK tiles, short enough that every workgroup gets work on small jobs
    const uint64_t per_wg = units / (grid ? grid : 1);
    const uint64_t run = ZF_CHUNK / ki.u;
    a.chunk = per_wg < 1 ? 1 : (per_wg < run ? per_wg : run);
    if (bl) {  // wave-level runs of 1 KiB units
        const uint64_t per_wave = (L.C / 1024) * L.count / (4 * (grid ? grid : 1));
        a.chunk = per_wave < 1 ? 1 : (per_wave < ZF_BL_RUN ? per_wave : ZF_BL_RUN);
    }
    if (L.pattern_only) {  // the product's grid, run length and LDS footprint; no arithmetic
        if (bl) return hipErrorInvalidValue;
        if (p.k == 4 && ng == 1 && ki.u == 2) fn = hbm_pattern_kernel<4, 4, 2, ZF_NT>;
        else if (p.k == 8 && ng == 2 && ki.u == 1) fn = hbm_pattern_kernel<8, 8, 1, false>;
        else return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(TPB), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

// The stream's run-queue block for other persistent kernels (K13 uses words
// 512 and 544, clear of K1's counters; each launch leaves its words zero).
hipError_t stream_queue(hipStream_t stream, uint32_t **out) { return queue_for(stream, out); }

void stream_queue_release(hipStream_t stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    const int dev = selected_device();
    auto it = g_queue.find(std::make_pair(dev, stream));
    if (it == g_queue.end()) return;
    g_queue_free[dev].push_back(it->second);
    g_queue.erase(it);
}

hipError_t zfec_parity_table(uint32_t k, uint32_t m, const void **out) {
    if (k == 0 || m <= k || m - k > 4) return hipErrorInvalidValue;
    const std::vector<uint8_t> enc = zfec_enc_matrix(k, m);
    GfPlan p;
    p.k = k;
    p.np = m - k;
    p.coef.assign(enc.begin() + (size_t)k * k, enc.end());
    return device_table(p, 1, out);
}

hipError_t gf_apply(const GfPlan &p, const GfLaunch &L, hipStream_t stream) {
    if (L.count == 0 || L.C == 0) return hipSuccess;
    KernelInfo fast;  // the fast kernel is instantiated for k in 1..8 and 16; other k take the generic one
    if (p.k > (uint32_t)ZF_MAXK || !lookup_fast((int)p.k, 1, fast)) {
        if (L.bao_off) return hipErrorInvalidValue;  // the bao-layout store exists for 4-of-8 only
        return apply_generic(p, L, stream);
    }
    if (p.np == 0) return gf_apply_pass(p, L, stream, 0, 0, true);
    for (uint32_t row0 = 0; row0 < p.np; row0 += ZF_MAXP) {
        const uint32_t nrows = p.np - row0 < (uint32_t)ZF_MAXP ? p.np - row0 : (uint32_t)ZF_MAXP;
        hipError_t e = gf_apply_pass(p, L, stream, row0, nrows, row0 == 0);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace chip

