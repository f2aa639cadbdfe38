// layout_store.hpp — whole-line stores of 1 KiB chunks into their bao slots.
//
// Used by the zfec kernel that writes encode()'s shards straight into the bao
// stream (zfec_device.hpp, gf_apply_bl_kernel).  Slots sit at 8 (mod 64) in the
// stream, so a chunk spans 9 memory lines; a 128-B line written in pieces by
// several store instructions costs far more than one written whole
// (tools/layout_probe.hip: 13.6 vs 11.1 ms per 1024 x 16 MiB of shards), so
// every line is written by ONE store instruction wherever its bytes are known:
//  * store A: the 8 lines [L0, L0 + 1024), L0 = the line holding the slot
//    start d; lane l = stream bytes [L0 + 16 l, +16).  Chunk bytes come from a
//    lane rotation by (d - L0)/16 (ds_bpermute); the bytes before d are the
//    chunk's parent slots (written as zeros: the bao kernels fill them later)
//    and, before those, the previous chunk's tail, which the previous chunk's
//    rotation left in the same lanes (`Spill`, kept in registers by a wave
//    that stores consecutive chunks);
//  * store B: the spill line [L0 + 1024, +128) with the chunk's last d - L0
//    bytes: written here when the rest of it is parent slots (zeros), else by
//    the next chunk's store A when the same wave stores that chunk next.
// Only where a wave's run of consecutive chunks starts or ends is a line
// written in two parts.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace chip {
namespace lay {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// chunk-slot offset tables are read through the constant address space:
// scalar loads, which never wait on the wave's outstanding stores
typedef const __attribute__((address_space(4))) uint64_t *ctab_t;

template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    else *reinterpret_cast<u32x4 *>(p) = v;
}

template <bool NT>
__device__ __forceinline__ void st8(uint8_t *p, u32x2 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x2 *>(p));
    else *reinterpret_cast<u32x2 *>(p) = v;
}

__device__ __forceinline__ uint32_t bperm(int src_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

struct Spill {  // the previous chunk's rotated data (its spill line in lanes 0..7)
    u32x2 lo, hi;
};

// Store full chunk ci (lane l holds chunk bytes [16 l, +16) in v) of a stream
// at ob whose N chunk slots are tab[0..N).  prev_ok: this wave stored chunk
// ci - 1 just before (sp holds its spill); next_ok: it stores chunk ci + 1
// next (and that chunk is a full one).  Updates sp for the next call.
template <bool NT>
__device__ __forceinline__ void put_chunk(uint8_t *ob, ctab_t tab, uint64_t N, uint64_t ci, const u32x4 &v,
                                          bool prev_ok, bool next_ok, Spill &sp) {
    const int lane = threadIdx.x & 63;
    const u32x2 zero = {0u, 0u};
    const uint64_t off = tab[ci];
    uint8_t *d = ob + off;
    const int r = (int)((uintptr_t)d & 127);
    uint8_t *L0 = d - r;
    const bool last = ci + 1 >= N;
    const int pb = ci == 0 ? 0 : (int)(off - tab[ci - 1] - 1024);  // parent bytes before the slot
    const uint64_t cnext = last ? 0 : (tab[ci + 1] - off - 1024) >> 6;
    // bytes [L0, d): parent slots only (zeros)?  else, before the parents, the
    // previous chunk's tail (chunk 0: never touched -- header / another stream)
    const bool pre_zero = ci != 0 && pb >= r;
    const bool pred_in = ci != 0 && !pre_zero && prev_ok;
    const bool post_zero = !last && 64 * cnext >= (uint64_t)(128 - r);
    const bool succ_takes = !last && !post_zero && next_ok;
    // rotation: lane l gets chunk bytes [16 l - r, +16) (mod 1024)
    const int rr = r >> 3;
    const int src0 = ((2 * lane - rr) >> 1) & 63, src1 = ((2 * lane - rr + 1) >> 1) & 63;
    const bool up0 = rr & 1;
    u32x2 lo, hi;
    lo.x = bperm(src0, up0 ? v.z : v.x);
    lo.y = bperm(src0, up0 ? v.w : v.y);
    hi.x = bperm(src1, up0 ? v.x : v.z);
    hi.y = bperm(src1, up0 ? v.y : v.w);
    const int b0 = 16 * lane - r, b1 = b0 + 8;  // chunk byte of each 8-B half of store A
    // store A; the previous chunk's spill line == this L0 exactly when it was
    // left to us, and its rotation holds those bytes in these lanes
    u32x2 a0 = lo, a1 = hi;
    if (b0 < 0) a0 = (pred_in && b0 < -pb) ? sp.lo : zero;
    if (b1 < 0) a1 = (pred_in && b1 < -pb) ? sp.hi : zero;
    if (b0 >= 0 || pre_zero || pred_in) st16<NT>(L0 + 16 * lane, u32x4{a0.x, a0.y, a1.x, a1.y});
    else if (b1 >= 0) st8<NT>(L0 + 16 * lane + 8, a1);
    // store B: chunk bytes 1024 + b0, 1024 + b1 (< 1024: this chunk's tail)
    if (r && lane < 8 && !succ_takes) {
        const bool in0 = b0 < 0, in1 = b1 < 0;
        uint8_t *q = L0 + 1024 + 16 * lane;
        if (in1 || post_zero)
            st16<NT>(q, u32x4{in0 ? lo.x : 0u, in0 ? lo.y : 0u, in1 ? hi.x : 0u, in1 ? hi.y : 0u});
        else if (in0)
            st8<NT>(q, lo);
    }
    sp.lo = lo;
    sp.hi = hi;
}

// Wave-level schedule of the layout kernels: XCD-grouped runs of CH
// consecutive units per wave (waves of one XCD, b % 8, take consecutive runs).
struct WaveRuns {
    uint64_t run, t_in, CH, GW, T;
    __device__ WaveRuns(uint64_t total, uint64_t ch) : t_in(0), CH(ch < 1 ? 1 : ch), T(total) {
        const uint64_t G = gridDim.x, b = blockIdx.x;
        const uint64_t w = (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const uint64_t wpb = blockDim.x / 64;
        GW = G * wpb;
        run = (G & 7) ? b * wpb + w : ((b % 8) * (G / 8) + b / 8) * wpb + w;
    }
    __device__ bool next(uint64_t &t) {
        if (t_in == CH) { run += GW; t_in = 0; }
        t = run * CH + t_in;
        ++t_in;
        return t < T;
    }
};

}  // namespace lay
}  // namespace chip
