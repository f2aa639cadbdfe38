// zfec_device.hpp — device code of K1/K2 (GF(2^8) stripe matrix-apply),
// shared by the product (zfec_kernels.hip) and tools/zfec_tune.hip.
// See zfec_kernels.hip for the design notes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "chip_internal.hpp"
#include "layout_store.hpp"

namespace chip {
namespace zf {

constexpr int TPB = 256;
constexpr int VEC = 16;
constexpr int TILE = TPB * VEC;  // byte-columns per workgroup tile

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct ApplyArgs {
    const uint8_t *in;
    uint8_t *out;
    uint64_t in_stride, out_stride, valid, C;
    uint64_t tiles_per_obj, total_tiles, count;
    uint64_t chunk;                    // MAP 3: tiles per XCD-grouped run (>= 1)
    const void *table;                 // [K][256] entries of NG dwords
    const uint64_t *bao_off;           // BL: stream offset of each 1 KiB chunk of the shard-major output
    uint64_t bao_n;                    // BL: number of chunks (bao_off entries)
    uint64_t in_off[ZF_MAXK];
    uint64_t copy_off[ZF_MAXK];
    uint64_t par_off[ZF_MAXP];
    uint32_t *queue;                   // MAP 6/7: run counters (QueueIter), zero at launch, left zero
    uint32_t xcd_mask;                 // MAP 6/7: XCDs whose workgroups take runs (0 = all)
    uint64_t *trace;                   // TR: per-workgroup {start, end, xcc, tiles} (tools only)
};

// Hardware XCC (XCD) id of the executing workgroup (gfx940+ HW_REG_XCC_ID).
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }

// Dynamic run queue (MAP 6 and 7).  The tile space is cut into runs of CH
// consecutive tiles, the runs into 8 shares, one per XCD.  A workgroup takes
// the next run of its own XCD's share (one device-scope atomic per run, by
// thread 0, broadcast through LDS) and, once that share is exhausted, runs
// of the following XCDs' shares: the XCDs that stream faster finish the
// slower ones' work instead of idling at the end of the launch.
//   MAP 6: share x = the x-th contiguous eighth of the runs;
//   MAP 7: MAP 3's interleave (the XCD's G/8 workgroups' runs of each
//          round of G runs), so all XCDs sweep one window of the batch.
// q[32 x] = run counter of share x, q[256] = workgroups done; the last
// workgroup to finish zeroes them, so every launch finds them zero.
template <int MAP>
struct QueueIter {
    uint32_t *q, *slot;
    uint64_t R, T, CH, g, run = 0, t_in = 0, rl = 0;
    uint32_t xcc, v = 0, k = 0;
    __device__ QueueIter(uint64_t total, uint64_t ch, uint32_t *queue, uint32_t *lds_slot, uint32_t mask)
        : q(queue), slot(lds_slot), T(total), CH(ch < 1 ? 1 : ch) {
        R = (T + CH - 1) / CH;
        g = gridDim.x / 8 ? gridDim.x / 8 : 1;
        xcc = xcc_id();
        if (mask && !((mask >> xcc) & 1u)) v = 8;  // this XCD sits out: the others take its share
    }
    // run index of the i-th run of share x, or ~0 past its end
    __device__ uint64_t share_run(uint32_t x, uint64_t i) const {
        if (MAP == 6) {
            const uint64_t lo = x * R / 8, hi = (x + 1) * R / 8;
            return lo + i < hi ? lo + i : ~0ull;
        }
        const uint64_t r = (i / g) * (8 * g) + x * g + (i % g);
        return r < R ? r : ~0ull;
    }
    __device__ bool grab() {
        uint32_t *s = slot + (k++ & 1);  // double-buffered: one barrier per grab
        if (threadIdx.x == 0) {
            uint32_t got = ~0u;
            while (v < 8) {
                const uint32_t x = (xcc + v) & 7u;
                const uint32_t i = atomicAdd(q + 32 * x, 1u);
                const uint64_t r = share_run(x, i);
                if (r != ~0ull) { got = (uint32_t)r; break; }
                ++v;
            }
            *s = got;
        }
        __syncthreads();
        const uint32_t r = *s;
        if (r == ~0u) return false;
        run = r;
        t_in = 0;
        rl = (run + 1) * CH <= T ? CH : T - run * CH;
        return true;
    }
    __device__ bool next(uint64_t &t) {
        if (t_in == rl && !grab()) return false;
        t = run * CH + t_in++;
        return true;
    }
    // every workgroup, after its last next(): the last one resets the counters
    __device__ void finish() {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(q + 256, 1u) == gridDim.x - 1) {
                for (int x = 0; x < 8; ++x) atomicExch(q + 32 * x, 0u);
                atomicExch(q + 256, 0u);
            }
        }
    }
};

__host__ __device__ constexpr int replicas_for(int k) {
    int r = 1;
    while (r * 2 * k <= 32) r *= 2;
    return r;
}

template <int NG> struct Entry;
template <> struct Entry<1> { using T = uint32_t; };
template <> struct Entry<2> { using T = u32x2; };

// 16 bytes at base+off with bytes at or past `valid` zeroed.  base+off is
// 16-B aligned (the C-ABI requires aligned pointers and strides), so the
// aligned block holding any valid byte lies inside a mapped page: one vector
// load + a byte mask, no byte-wise loads (they inflated K=8 to 350+ VGPRs).
template <bool NTL = false>
__device__ __forceinline__ u32x4 load16_masked(const uint8_t *base, uint64_t off, uint64_t valid) {
    if (off >= valid) return u32x4{0u, 0u, 0u, 0u};
    u32x4 r = NTL ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + off))
                  : *reinterpret_cast<const u32x4 *>(base + off);
    if (off + VEC > valid) {
        const int rem = (int)(valid - off);  // 1..15
        auto keep = [rem](int i) -> uint32_t {
            const int b = rem - 4 * i;
            return b >= 4 ? ~0u : b <= 0 ? 0u : ((1u << (8 * b)) - 1u);
        };
        r.x &= keep(0); r.y &= keep(1); r.z &= keep(2); r.w &= keep(3);
    }
    return r;
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t *p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    else *reinterpret_cast<u32x4 *>(p) = v;
}

template <bool NT>
__device__ __forceinline__ void store8z(uint8_t *p, u32x2 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x2 *>(p));
    else *reinterpret_cast<u32x2 *>(p) = v;
}

// Store the 16 B of output byte offset p (shard-major layout).
template <bool NT>
__device__ __forceinline__ void put16(uint8_t *ob, uint64_t p, u32x4 v) {
    store16<NT>(ob + p, v);
}

// rows[q] = byte q of a0..a3 (4x4 byte transpose, 8 v_perm_b32)
__device__ __forceinline__ void transpose4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                           uint32_t &r0, uint32_t &r1, uint32_t &r2, uint32_t &r3) {
    const uint32_t u0 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);  // a0b0 a1b0 a0b1 a1b1
    const uint32_t u1 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);  // a0b2 a1b2 a0b3 a1b3
    const uint32_t w0 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
    const uint32_t w1 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
    r0 = __builtin_amdgcn_perm(w0, u0, 0x05040100u);
    r1 = __builtin_amdgcn_perm(w0, u0, 0x07060302u);
    r2 = __builtin_amdgcn_perm(w1, u1, 0x05040100u);
    r3 = __builtin_amdgcn_perm(w1, u1, 0x07060302u);
}

__device__ __forceinline__ uint32_t comp(const u32x4 &v, int d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Tile schedule (MAP), per workgroup b of G:
//   0  grid-stride: tile = b, b + G, b + 2G, ...
//   1  XCD-grouped grid-stride: the G/8 workgroups that share an XCD
//      (b % 8, observed round-robin dispatch; speed only, never correctness)
//      take G/8 consecutive tiles each round
//   2  one contiguous range per workgroup
//   3  XCD-grouped chunks: runs of CH consecutive tiles dealt as in 1, each
//      run walked in order by one workgroup (long sequential streams per
//      shard; tools/write_probe: HBM writes 5.0 -> 5.9 TB/s)
//   5  as 3, each workgroup starting its runs at its own rotated tile (a
//      per-workgroup offset mod CH, wrapping inside the run).  Runs begin at
//      multiples of CH tiles in every object and shard, so under 3 all
//      workgroups advance in lockstep at the same offset inside their runs
//      and every stream in flight shares the same low address bits.
// Falls back to 0 when G is not a multiple of 8.
template <int MAP>
struct TileIter {
    uint64_t T, c, t_in, end, stride, base, CH;
    uint64_t rot = 0, rl = 0, rotr = 0;  // MAP 5: rotation, current run length, rotation mod rl
    int mode;
    __device__ void start_run() {
        rl = c * CH >= T ? 0 : (T - c * CH < CH ? T - c * CH : CH);
        rotr = rl == CH ? rot : (rl ? rot % rl : 0);
    }
    __device__ TileIter(uint64_t total, uint64_t ch) : T(total), t_in(0), CH(ch < 1 ? 1 : ch) {
        const uint64_t G = gridDim.x, b = blockIdx.x;
        mode = ((MAP == 1 || MAP == 3 || MAP == 5) && (G & 7)) ? 0 : MAP;
        if (mode == 2) {
            const uint64_t chunk = (T + G - 1) / G;
            c = b * chunk;
            end = c + chunk < T ? c + chunk : T;
            stride = 1;
            base = 0;
        } else if (mode == 1 || mode == 3 || mode == 5) {
            base = (b % 8) * (G / 8) + b / 8;
            c = base;
            stride = G;
            end = T;
            if (mode == 5) {
                rot = (b * 37 + (b >> 3)) % CH;
                start_run();
            }
        } else {
            c = b;
            stride = G;
            end = T;
            base = 0;
        }
    }
    __device__ bool next(uint64_t &t) {
        if (mode == 5) {
            if (t_in == rl) {
                c += stride;
                t_in = 0;
                start_run();
            }
            if (rl == 0) return false;
            uint64_t i = t_in + rotr;
            if (i >= rl) i -= rl;
            t = c * CH + i;
            ++t_in;
            return true;
        }
        if (mode == 3) {
            if (t_in == CH) { c += stride; t_in = 0; }
            t = c * CH + t_in;
            ++t_in;
            return t < T;
        }
        t = c;
        c += stride;
        return t < end;
    }
};

// The kernel body.  RO: replica-count override, WPE: waves/EU hint, SB:
// scheduling fence every SB shards (bounds the table lookups in flight; 0 =
// none), PF: load the next super-tile's shards before computing the current
// one, NTL: nontemporal input loads, TR: per-workgroup trace — tools/zfec_tune.
// The product's kernels are zfec_kernels.hip's zfec_apply_kernel<K, NG> (one
// configuration per shape, ApplyCfg); the tuner's, tools/zfec_variants.hpp's.
template <int K, int NG, int U, int MAP, bool NT, int RO = 0, int WPE = 1, int SB = 0, bool PF = false,
          bool NTL = false, bool TR = false>
__device__ __forceinline__ void gf_apply_body(const ApplyArgs &a) {
    constexpr int R = RO ? RO : replicas_for(K);
    using E = typename Entry<NG>::T;
    constexpr int W = 4 * NG;            // bytes per table entry
    constexpr int ROWB = K * R * W;      // bytes per table row (one byte value x)
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];

    // ---- table fill: lds[x][s][r] = T_s[x] ----
    {
        const E *tab = reinterpret_cast<const E *>(a.table);
        E *dst = reinterpret_cast<E *>(lds);
        for (int i = threadIdx.x; i < 256 * K * R; i += TPB) {
            const int x = i / (K * R);
            const int s = (i - x * (K * R)) / R;
            dst[i] = tab[s * 256 + x];
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int r = lane % R;
    const int grp = (lane & 31) / R;
    uint32_t tb[K];
    uint64_t ioff[K], coff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int s = (j + grp) % K;
        tb[j] = (uint32_t)((s * R + r) * W);
        ioff[j] = a.in_off[s];
        coff[j] = a.copy_off[s];
    }

    // super-tiles of U adjacent column tiles of one object
    const uint64_t spo = (a.tiles_per_obj + U - 1) / U;
    uint64_t t_start = 0, n_tiles = 0;
    if constexpr (TR) t_start = wall_clock64();
    __shared__ uint32_t q_slot[2];
    using Iter = typename std::conditional<(MAP >= 6), QueueIter<MAP>, TileIter<MAP>>::type;
    Iter iter = [&] {
        if constexpr (MAP >= 6) return Iter(spo * a.count, a.chunk, a.queue, q_slot, a.xcd_mask);
        else return Iter(spo * a.count, a.chunk);
    }();
    auto load_tile = [&](uint64_t t, u32x4 (&v)[U][K]) {
        const uint64_t obj = t / spo;
        const uint64_t col0 = (t - obj * spo) * (uint64_t)(U * TILE) + threadIdx.x * VEC;
        const uint8_t *ib = a.in + obj * a.in_stride;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint64_t col = col0 + (uint64_t)u * TILE;
                v[u][j] = col < a.C ? load16_masked<NTL>(ib, ioff[j] + col, a.valid) : u32x4{0u, 0u, 0u, 0u};
            }
    };

    uint64_t st;
    bool have = iter.next(st);
    u32x4 v[U][K];
    if (PF && have) load_tile(st, v);
    while (have) {
        uint64_t st_next;
        const bool have_next = iter.next(st_next);
        u32x4 vn[U][K];
        if constexpr (PF) {
            if (have_next) load_tile(st_next, vn);
        } else {
            load_tile(st, v);
        }
        const uint64_t obj = st / spo;
        const uint64_t col0 = (st - obj * spo) * (uint64_t)(U * TILE) + threadIdx.x * VEC;
        uint8_t *ob = a.out + obj * a.out_stride;

#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t col = col0 + (uint64_t)u * TILE;
            if (col >= a.C) continue;
            // acc[c] = packed computed-row bytes of byte-column c (16 columns)
            E acc[16];
#pragma unroll
            for (int j = 0; j < K; ++j) {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t x = comp(v[u][j], d);
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t byte = (x >> (8 * b)) & 0xFFu;
                        const E e = *reinterpret_cast<const E *>(lds + byte * ROWB + tb[j]);
                        if (j == 0) acc[d * 4 + b] = e;
                        else acc[d * 4 + b] ^= e;
                    }
                }
                // Pin the partial sums every SB shards: otherwise LLVM's
                // reassociation rebuilds each K-term XOR chain at its root, so
                // all K*16 lookups are live at once (K=8: 350+ VGPRs, spills).
                if constexpr (SB > 0)
                    if ((j + 1) % SB == 0 && j + 1 < K) {
#pragma unroll
                        for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(acc[c]));
                    }
            }

            // copies (data shards for encode, surviving primaries for decode)
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (coff[j] != NO_OUT) store16<NT>(ob + coff[j] + col, v[u][j]);

            // computed rows: transpose column-packed sums into row streams
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                uint32_t rows[4][4];  // [q][d]
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t c0, c1, c2, c3;
                    if constexpr (NG == 1) {
                        c0 = acc[d * 4 + 0]; c1 = acc[d * 4 + 1]; c2 = acc[d * 4 + 2]; c3 = acc[d * 4 + 3];
                    } else {
                        c0 = acc[d * 4 + 0][g]; c1 = acc[d * 4 + 1][g];
                        c2 = acc[d * 4 + 2][g]; c3 = acc[d * 4 + 3][g];
                    }
                    transpose4(c0, c1, c2, c3, rows[0][d], rows[1][d], rows[2][d], rows[3][d]);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint64_t po = a.par_off[g * 4 + q];
                    if (po == NO_OUT) continue;
                    u32x4 o = {rows[q][0], rows[q][1], rows[q][2], rows[q][3]};
                    put16<NT>(ob, po + col, o);
                }
            }
        }
        if constexpr (PF) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < K; ++j) v[u][j] = vn[u][j];
        }
        st = st_next;
        have = have_next;
        if constexpr (TR) ++n_tiles;
    }
    if constexpr (MAP >= 6) iter.finish();
    if constexpr (TR) {
        if (threadIdx.x == 0) {
            uint64_t *tr = a.trace + 4 * blockIdx.x;
            tr[0] = t_start;
            tr[1] = wall_clock64();
            tr[2] = xcc_id();
            tr[3] = n_tiles;
        }
    }
}

// BL (bao layout, encode() with Zfec|Bao): zfec 4-of-8 encode whose 8 output
// shards go straight into their chunk slots of each object's bao stream
// (shard byte p at bao_off[p >> 10] + (p & 1023)), every memory line written
// whole by one store where its bytes are known (layout_store.hpp).  A unit is
// one 1 KiB chunk-column (the same 1 KiB of columns of every shard); a WAVE
// walks runs of consecutive units on its own (no workgroup barrier: the 4
// waves of a workgroup share only the LDS table), so the chunk before a
// chunk, in every shard, is the wave's previous unit and its spill bytes are
// still in registers.  The next unit's 4 data-shard loads are in flight while
// a unit is computed.
// BL = false: the same wave-private schedule writing the plain shard-major
// layout (a K1 variant for tools/zfec_tune).
template <bool NT, bool BL = true>
__global__ __launch_bounds__(TPB) void gf_apply_bl_kernel(ApplyArgs a) {
    constexpr int K = 4, R = replicas_for(4), W = 4, ROWB = K * R * W;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    {
        const uint32_t *tab = reinterpret_cast<const uint32_t *>(a.table);
        uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
        for (int i = threadIdx.x; i < 256 * K * R; i += TPB) {
            const int x = i / (K * R);
            const int s = (i - x * (K * R)) / R;
            dst[i] = tab[s * 256 + x];
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int rep = lane % R, grp = (lane & 31) / R;
    uint32_t tb[K];
    uint64_t ioff[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        tb[j] = (uint32_t)((((j + grp) % K) * R + rep) * W);
        ioff[j] = a.in_off[(j + grp) % K];
    }

    const uint64_t Cc = a.C >> 10;  // units (chunk-columns) per object
    lay::WaveRuns runs(Cc * a.count, a.chunk);
    auto load_unit = [&](uint64_t t, u32x4 (&v)[K]) {
        const uint64_t obj = t / Cc;
        const uint64_t col = (t - obj * Cc) * 1024 + lane * 16;
        const uint8_t *ib = a.in + obj * a.in_stride;
#pragma unroll
        for (int j = 0; j < K; ++j) v[j] = load16_masked(ib, ioff[j] + col, a.valid);
    };
    const lay::ctab_t tab = (lay::ctab_t)a.bao_off;
    lay::Spill spill[8];  // the previous unit's spill lines, per shard
    uint64_t prev_t = ~0ull;
    uint64_t t;
    bool have = runs.next(t);
    u32x4 v[K];
    if (have) load_unit(t, v);
    while (have) {
        uint64_t tn;
        const bool have_next = runs.next(tn);
        u32x4 vn[K];
        if (have_next) load_unit(tn, vn);
        const uint64_t obj = t / Cc, uc = t - obj * Cc;
        uint8_t *ob = a.out + obj * a.out_stride;
        const bool prev_ok = prev_t + 1 == t && uc > 0;                  // the previous chunk, every shard
        const bool next_ok = have_next && tn == t + 1 && uc + 1 < Cc;   // the next chunk, every shard

        uint32_t acc[16];
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
            for (int dd = 0; dd < 4; ++dd) {
                const uint32_t x = comp(v[j], dd);
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                    const uint32_t e = *reinterpret_cast<const uint32_t *>(lds + ((x >> (8 * bb)) & 0xFFu) * ROWB + tb[j]);
                    if (j == 0) acc[dd * 4 + bb] = e;
                    else acc[dd * 4 + bb] ^= e;
                }
            }
        }
        u32x4 ov[8];  // this lane's 16 B of every output shard, shard order
#pragma unroll
        for (int sh = 0; sh < K; ++sh) {
            const int jj = (sh - grp + K) % K;
            u32x4 x = v[0];
#pragma unroll
            for (int j = 1; j < K; ++j)
                if (jj == j) x = v[j];
            ov[sh] = x;
        }
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
            uint32_t r0, r1, r2, r3;
            transpose4(acc[dd * 4 + 0], acc[dd * 4 + 1], acc[dd * 4 + 2], acc[dd * 4 + 3], r0, r1, r2, r3);
            if (dd == 0) { ov[4].x = r0; ov[5].x = r1; ov[6].x = r2; ov[7].x = r3; }
            if (dd == 1) { ov[4].y = r0; ov[5].y = r1; ov[6].y = r2; ov[7].y = r3; }
            if (dd == 2) { ov[4].z = r0; ov[5].z = r1; ov[6].z = r2; ov[7].z = r3; }
            if (dd == 3) { ov[4].w = r0; ov[5].w = r1; ov[6].w = r2; ov[7].w = r3; }
        }

        if constexpr (BL) {
#pragma unroll
            for (int sh = 0; sh < 8; ++sh)
                lay::put_chunk<NT>(ob, tab, a.bao_n, (uint64_t)sh * Cc + uc, ov[sh], prev_ok, next_ok, spill[sh]);
        } else {
#pragma unroll
            for (int sh = 0; sh < 8; ++sh) store16<NT>(ob + (uint64_t)sh * a.C + uc * 1024 + lane * 16, ov[sh]);
        }
        prev_t = t;
#pragma unroll
        for (int j = 0; j < K; ++j) v[j] = vn[j];
        t = tn;
        have = have_next;
    }
}

}  // namespace zf
}  // namespace chip
