// quad_b3.hpp — BLAKE3 compression on four lanes (a quad), shared by KS
// (small_kernels.hip: one workgroup per small object) and KM
// (multi_kernels.hip: one single object over many workgroups).
//
// Lane q of a quad holds column q of the BLAKE3 state (a, b, c, d) and runs
// that column's G; the diagonal step rotates b, c, d across the quad with DPP
// quad permutes and back.  7 rounds of 2 G (12 ops each) and 6 DPP moves:
// ~220 VALU per compression per lane instead of ~700 for one lane alone.  The
// message words a lane needs in round r are m[SCHED(r, 2q)], m[SCHED(r, 2q + 1)]
// (column) and m[SCHED(r, 8 + 2q)], m[SCHED(r, 9 + 2q)] (diagonal), read from
// the quad's 64-B LDS slot at per-lane offsets fixed at kernel start.
#pragma once

#include "bao_device.hpp"

namespace chip {
namespace small {

using namespace bao;

// value of x held by lane (q + K) & 3 of my quad
template <int K>
__device__ __forceinline__ uint32_t qrot(uint32_t x) {
    constexpr int ctrl = K == 1 ? 0x39 : K == 2 ? 0x4E : 0x93;  // quad_perm [1,2,3,0] / [2,3,0,1] / [3,0,1,2]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, false);
}

// Per-lane LDS byte offsets of the message words of each round (within the
// quad's slot): [r][0..1] column G, [r][2..3] diagonal G.
struct MsgIdx {
    uint32_t o[28];
    __device__ explicit MsgIdx(int q, uint32_t slot) {
#pragma unroll
        for (int r = 0; r < 7; ++r) {
            uint32_t c0 = 0, c1 = 0, d0 = 0, d1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (q == k) {
                    c0 = SCHED(r, 2 * k); c1 = SCHED(r, 2 * k + 1);
                    d0 = SCHED(r, 8 + 2 * k); d1 = SCHED(r, 9 + 2 * k);
                }
            o[4 * r] = slot + 4 * c0; o[4 * r + 1] = slot + 4 * c1;
            o[4 * r + 2] = slot + 4 * d0; o[4 * r + 3] = slot + 4 * d1;
        }
    }
};

__device__ __forceinline__ uint32_t lds_word(const uint8_t *lds, uint32_t off) {
    return *reinterpret_cast<const uint32_t *>(lds + off);
}

// (h0, h1) = words q and 4 + q of the CV, updated to compress(h, m, ctr,
// blen, flags) with the message in the quad's LDS slot.
__device__ __forceinline__ void compress4(uint32_t &h0, uint32_t &h1, const uint8_t *lds, const MsgIdx &mi,
                                          int q, uint32_t ivq, uint64_t ctr, uint32_t blen, uint32_t flags) {
    uint32_t m[28];
#pragma unroll
    for (int i = 0; i < 28; ++i) m[i] = lds_word(lds, mi.o[i]);
    uint32_t a = h0, b = h1, c = ivq;
    uint32_t d = q == 0 ? (uint32_t)ctr : q == 1 ? (uint32_t)(ctr >> 32) : q == 2 ? blen : flags;
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        B3G(a, b, c, d, m[4 * r], m[4 * r + 1]);
        b = qrot<1>(b); c = qrot<2>(c); d = qrot<3>(d);
        B3G(a, b, c, d, m[4 * r + 2], m[4 * r + 3]);
        b = qrot<3>(b); c = qrot<2>(c); d = qrot<1>(d);
    }
    h0 = a ^ c;
    h1 = b ^ d;
}

__device__ __forceinline__ u32x4 load16_bytes(const uint8_t *p, uint32_t valid) {  // valid < 16: byte loads
    return valid == 0 ? u32x4{0u, 0u, 0u, 0u} : load16_partial(p, valid);
}

}  // namespace small
}  // namespace chip
