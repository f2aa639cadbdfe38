// small_kernels.hip — KS: one workgroup encodes or verify-decodes one small
// object (bao stream of N <= 512 chunks) in one launch (gfx950).
//
// The batch kernels (K13, K3 + K4/K4t) are built for throughput: one lane
// hashes a whole 1 KiB chunk (16 dependent BLAKE3 compressions of ~700 VALU
// instructions each, ~19 us for one wave), and a call runs two or more
// launches.  A single small object through them costs 40-50 us of kernel
// time for one chunk (profiles/r4c).  KS is built for latency instead:
//
//  * four lanes share one compression: lane q of a quad holds column q of the
//    BLAKE3 state (a, b, c, d) and runs that column's G; the diagonal step
//    rotates b, c, d across the quad with DPP quad permutes and back.  7 rounds
//    of 2 G (12 ops each) and 6 DPP moves: ~220 VALU per compression per
//    lane instead of ~700, so a chunk's 16 compressions take about a third of
//    the time.  The message words a lane needs in round r are
//    m[SCHED(r, 2q)], m[SCHED(r, 2q + 1)] (column) and m[SCHED(r, 8 + 2q)],
//    m[SCHED(r, 9 + 2q)] (diagonal): read from the quad's 64-B LDS slot at
//    per-lane offsets fixed at kernel start.
//  * one launch does everything: (encode) the header, the zfec shards or the
//    content into their chunk slots, the chunk CVs, every parent level (K4t's
//    level walk, CVs in LDS, each parent also on four lanes) and the root
//    hash; (decode) the content prefix out, every chunk and parent recomputed
//    and compared with the stored node, the root with the expected hash.
//
// Used for single-object calls (count == 1, N <= KS_MAX_N) and for batches
// of tiny objects (N <= KS_TINY_N) of bao encode / decode and encode() at
// Zfec|Bao; CHIP_SMALL=0 turns it off (A/B runs and tests compare the paths
// byte for byte).
#include "bao_device.hpp"
#include "chip_internal.hpp"
#include "quad_b3.hpp"
#include "zfec_device.hpp"

#include <cstdlib>
#include <cstring>

namespace chip {

using namespace bao;

namespace small {

// Two shapes: one object per call (512 threads = 128 quads, N <= 512: one
// chunk round for up to 128 chunks) and batches of tiny objects (64 threads =
// 16 quads, N <= 64: one wave per object, so a CU holds many objects at once
// where the batch kernels would run 1-8 of a wave's 64 lanes).
constexpr int BIG_TPB = 512, BIG_N = 512;
constexpr int TINY_TPB = 64, TINY_N = 64;
static_assert(BIG_N <= K4T_MAX, "tree walk bound");

struct SmallArgs {
    const uint8_t *in;      // encode: content (C == 0) or zfec input; decode: stream
    uint8_t *out;           // encode: stream (may be null when C == 0: hash only); decode: content
    uint64_t in_stride, out_stride;
    uint64_t n;             // bao content bytes (encode with zfec: 8 C)
    uint64_t N;             // chunks of the bao content
    uint64_t valid;         // encode with zfec: input bytes (zero beyond)
    uint64_t C;             // encode: zfec 4-of-8 shard length, 0 = bao of the content
    uint64_t out_limit;     // decode: content bytes written
    uint64_t count;
    uint32_t per;           // objects per workgroup (a power of two; per * N <= QUADS when > 1)
    const uint32_t *table;  // zfec parity table [4][256]
    uint8_t *hash;          // encode: root hashes out; decode: expected
    uint32_t *status;       // decode: per object, 0 or CHIP_ERR_BAO_HASH_MISMATCH
};

// MODE 0: encode, MODE 1: verify-decode.  A workgroup holds a.per objects
// (1 unless N is small enough for several to share the quads), N <= MAXN / per.
template <int MODE, int TPB, int MAXN>
__global__ __launch_bounds__(TPB) void small_kernel(SmallArgs a) {
    constexpr int QUADS = TPB / 4;
    __shared__ __attribute__((aligned(16))) uint32_t tab[4 * 256];     // zfec parity products
    __shared__ __attribute__((aligned(16))) uint32_t cvs[2][MAXN][8];  // one tree level and the next
    __shared__ __attribute__((aligned(16))) uint32_t msg[QUADS][16];  // each quad's message block
    // encode() at Zfec|Bao of one object of at most 64 chunks: the shards also
    // kept here, so phase 2 hashes them without reading back the stream (a
    // single call's stream is pinned host memory: a PCIe round trip)
    constexpr int STG = MODE == 0 && MAXN > 64 ? 64 * 64 : 1;  // 16-B units: 64 chunks
    __shared__ __attribute__((aligned(16))) u32x4 stg[STG];
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const int GT = TPB / (int)a.per, GQ = GT / 4;  // threads and quads of one object
    const int ol = t / GT, tl = t - ol * GT, gl = tl >> 2;
    const uint64_t obj = (uint64_t)blockIdx.x * a.per + ol;
    const bool live = obj < a.count;
    const uint32_t cb = (uint32_t)ol * (MAXN / a.per);  // my object's CV rows
    const uint64_t N = a.N, n = a.n;
    const uint8_t *src = a.in + (live ? obj : 0) * a.in_stride;
    uint8_t *dst = a.out ? a.out + (live ? obj : 0) * a.out_stride : nullptr;
    const uint8_t *stream = MODE == 0 ? dst : src;
    const bool staged = STG > 1 && a.C && N <= 64 && a.per == 1;
    bool ok = true;

    // ---- phase 1: header; zfec shards or content into their slots / content out
    if (MODE == 0) {
        if (live && dst && tl == 0) *glb(reinterpret_cast<uint64_t *>(dst)) = n;
        if (a.C) {
            for (int i = t; i < 4 * 256; i += TPB) tab[i] = a.table[i];
            __syncthreads();
            const uint64_t cols = a.C / 1024;
            for (uint64_t o = 16 * (uint64_t)tl; live && o < a.C; o += 16 * GT) {  // 16 B of every shard at byte o
                u32x4 v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = zf::load16_masked(src, j * a.C + o, a.valid);
                uint32_t acc[16];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        uint32_t x = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) x ^= tab[j * 256 + ((zf::comp(v[j], d) >> (8 * b)) & 0xFFu)];
                        acc[d * 4 + b] = x;
                    }
                }
                u32x4 p[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t r0, r1, r2, r3;
                    zf::transpose4(acc[d * 4], acc[d * 4 + 1], acc[d * 4 + 2], acc[d * 4 + 3], r0, r1, r2, r3);
                    if (d == 0) { p[0].x = r0; p[1].x = r1; p[2].x = r2; p[3].x = r3; }
                    if (d == 1) { p[0].y = r0; p[1].y = r1; p[2].y = r2; p[3].y = r3; }
                    if (d == 2) { p[0].z = r0; p[1].z = r1; p[2].z = r2; p[3].z = r3; }
                    if (d == 3) { p[0].w = r0; p[1].w = r1; p[2].w = r2; p[3].w = r3; }
                }
                const uint64_t u = o / 1024, w = o % 1024;
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    store16_a8<false>(dst + chunk_stream_off(s * cols + u, N) + w, s < 4 ? v[s] : p[s - 4]);
                    if (staged) stg[(s * cols + u) * 64 + w / 16] = s < 4 ? v[s] : p[s - 4];
                }
            }
        } else if (dst) {
            for (uint64_t o = 16 * (uint64_t)tl; live && o < n; o += 16 * GT) {
                const u32x4 v = zf::load16_masked(src, o, n);
                uint8_t *p = dst + chunk_stream_off(o / 1024, N) + o % 1024;
                if (o + 16 <= n) store16_a8<false>(p, v);
                else store16_partial(p, v, (uint32_t)(n - o));
            }
        }
    } else {
        if (live && tl == 0 && *reinterpret_cast<const uint64_t *>(src) != n) ok = false;
        for (uint64_t o = 16 * (uint64_t)tl; live && o < a.out_limit; o += 16 * GT) {
            const uint8_t *p = src + chunk_stream_off(o / 1024, N) + o % 1024;
            const uint64_t left = a.out_limit - o;
            if (left >= 16) {
                *glb(reinterpret_cast<u32x4 *>(dst + o)) = load16_a8(p);
            } else {
                store16_partial(dst + o, load16_bytes(p, (uint32_t)left), (uint32_t)left);
            }
        }
    }
    __syncthreads();  // (encode) the slots written above are read back below

    // ---- phase 2: chunk CVs, one quad per chunk
    const uint32_t slot = (uint32_t)(reinterpret_cast<uintptr_t>(&msg[g][0]) - reinterpret_cast<uintptr_t>(&msg[0][0]));
    const uint8_t *mbase = reinterpret_cast<const uint8_t *>(&msg[0][0]);
    const MsgIdx mi(q, slot);
    const uint32_t iv0 = q == 0 ? IV(0) : q == 1 ? IV(1) : q == 2 ? IV(2) : IV(3);
    const uint32_t iv1 = q == 0 ? IV(4) : q == 1 ? IV(5) : q == 2 ? IV(6) : IV(7);
    const bool content_in = MODE == 0 && a.C == 0;  // encode of the content: read it where it is
    // verify, one object per workgroup: the stored node of my first parent at
    // every level, in flight with my first chunk (one round of loads instead
    // of one dependent wait per level: a single call's stream is pinned host
    // memory, a PCIe round trip each).  Not in the tiny-batch shape, whose
    // occupancy the extra registers would cut (168 -> 206 VGPRs, 3 -> 2 waves)
    constexpr bool PF = MODE == 1 && MAXN > 64;
    constexpr int LOGMAX = 9;
    static_assert((1 << LOGMAX) >= MAXN, "levels of the walk");
    u32x4 stn[PF ? LOGMAX : 1];
    if (PF) {
        uint64_t cp_ = N;
#pragma unroll
        for (int l = 1; l <= LOGMAX; ++l) {
            const uint64_t cn = (cp_ + 1) / 2;
            stn[l - 1] = u32x4{0u, 0u, 0u, 0u};
            if (live && cp_ > 1 && (uint64_t)gl < cn && 2 * (uint64_t)gl + 1 < cp_)
                stn[l - 1] = load16_a8(src + parent_stream_off((uint64_t)gl << l, l, N) + 16 * q);
            cp_ = cn;
        }
    }
    for (uint64_t c = gl; live && c < N; c += GQ) {
        const uint64_t rem = n - c * 1024;
        const uint32_t clen = n == 0 ? 0u : (rem < 1024 ? (uint32_t)rem : 1024u);
        const uint32_t nb = clen == 0 ? 1u : (clen + 63) / 64;
        const uint8_t *cp = content_in ? src + c * 1024 : stream + chunk_stream_off(c, N);
        u32x4 pc[16];
#pragma unroll
        for (int b = 0; b < 16; ++b) {  // my 16 B of every block of the chunk, all loads in flight
            const uint32_t off = 64 * b + 16 * q;
            if (off >= clen) pc[b] = u32x4{0u, 0u, 0u, 0u};
            else if (staged) pc[b] = stg[c * 64 + off / 16];  // (zfec shards: whole chunks)
            else if (content_in) pc[b] = zf::load16_masked(src, c * 1024 + off, n);
            else pc[b] = off + 16 <= clen ? load16_a8(cp + off) : load16_bytes(cp + off, clen - off);
        }
        uint32_t h0 = iv0, h1 = iv1;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            if ((uint32_t)b < nb) {
                *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = pc[b];
                wave_sync();
                const bool last = (uint32_t)b + 1 == nb;
                const uint32_t flags = (b == 0 ? F_CHUNK_START : 0u) | (last ? F_CHUNK_END : 0u) |
                                       (last && N == 1 ? F_ROOT : 0u);
                compress4(h0, h1, mbase, mi, q, iv0, c, last ? clen - 64 * b : 64u, flags);
                wave_sync();
            }
        }
        if (N == 1) {  // the chunk is the root
            uint32_t *hp = reinterpret_cast<uint32_t *>(a.hash + obj * 32);
            if (MODE == 0) {
                hp[q] = h0;
                hp[4 + q] = h1;
            } else {
                ok &= hp[q] == h0 && hp[4 + q] == h1;
            }
        } else {
            cvs[0][cb + c][q] = h0;
            cvs[0][cb + c][4 + q] = h1;
        }
    }
    __syncthreads();

    // ---- phase 3: the parent levels (bao_top_kernel's walk), one quad per parent
    int cur = 0;
    uint64_t cnt_prev = N;
    for (int level = 1; cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        for (uint64_t p = gl; live && p < cnt; p += GQ) {
            if (2 * p + 1 >= cnt_prev) {  // odd last node: promoted unchanged
                cvs[cur ^ 1][cb + p][q] = cvs[cur][cb + 2 * p][q];
                cvs[cur ^ 1][cb + p][4 + q] = cvs[cur][cb + 2 * p][4 + q];
                continue;
            }
            // message = left CV || right CV: my 16 B are words 4q..4q+3
            const u32x4 mw = *reinterpret_cast<const u32x4 *>(&cvs[cur][cb + 2 * p + (q >> 1)][4 * (q & 1)]);
            *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = mw;
            wave_sync();
            const bool root = cnt == 1;
            uint32_t h0 = iv0, h1 = iv1;
            compress4(h0, h1, mbase, mi, q, iv0, 0, 64, F_PARENT | (root ? F_ROOT : 0u));
            wave_sync();
            uint8_t *node = const_cast<uint8_t *>(stream) + parent_stream_off(p << level, level, N) + 16 * q;
            if (MODE == 0) {
                if (dst) store16_a8<false>(node, mw);
            } else {
                u32x4 s;
                if (PF && p == (uint64_t)gl) {
                    s = stn[0];
#pragma unroll
                    for (int l = 2; l <= (PF ? LOGMAX : 1); ++l)
                        if (level == l) s = stn[l - 1];
                } else {
                    s = load16_a8(node);  // tiny batches; a quad's second parent of a level (N > 2 GQ)
                }
                ok &= s.x == mw.x && s.y == mw.y && s.z == mw.z && s.w == mw.w;
            }
            if (root) {
                uint32_t *hp = reinterpret_cast<uint32_t *>(a.hash + obj * 32);
                if (MODE == 0) {
                    hp[q] = h0;
                    hp[4 + q] = h1;
                } else {
                    ok &= hp[q] == h0 && hp[4 + q] == h1;
                }
            } else {
                cvs[cur ^ 1][cb + p][q] = h0;
                cvs[cur ^ 1][cb + p][4 + q] = h1;
            }
        }
        __syncthreads();
        cur ^= 1;
        cnt_prev = cnt;
    }
    if (MODE == 1 && live && !ok) flag_mismatch(a.status, obj);
}

bool enabled() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_SMALL");
        return !(e && !std::strcmp(e, "0"));
    }();
    return on;
}

hipError_t launch(int mode, SmallArgs a, hipStream_t stream) {
    if (a.count == 0) return hipSuccess;
    if (a.count > 0x7fffffffull) return hipErrorInvalidValue;
    const bool tiny = a.N <= (uint64_t)TINY_N && a.count > 1;
    a.per = 1;  // tiny objects: as many per workgroup as fill its 16 quads
    while (tiny && a.per * 2 * a.N <= (uint64_t)(TINY_TPB / 4) && a.per * 2 <= a.count) a.per *= 2;
    const dim3 grid((unsigned)((a.count + a.per - 1) / a.per));
    if (tiny) {
        if (mode == 0) hipLaunchKernelGGL((small_kernel<0, TINY_TPB, TINY_N>), grid, dim3(TINY_TPB), 0, stream, a);
        else hipLaunchKernelGGL((small_kernel<1, TINY_TPB, TINY_N>), grid, dim3(TINY_TPB), 0, stream, a);
    } else {
        if (mode == 0) hipLaunchKernelGGL((small_kernel<0, BIG_TPB, BIG_N>), grid, dim3(BIG_TPB), 0, stream, a);
        else hipLaunchKernelGGL((small_kernel<1, BIG_TPB, BIG_N>), grid, dim3(BIG_TPB), 0, stream, a);
    }
    return hipGetLastError();
}

// K4t for one object with a quad per parent (small_kernel's phase 3 over a
// level of cnt_prev <= K4T_MAX CVs): a single object's tree top is ~10
// dependent levels, latency-bound with a lane per parent (r10zm: 24-29 us of
// a 1 MiB call).  Same nodes, hash and verdict as bao_top_kernel.
template <int MODE>
__global__ __launch_bounds__(BIG_TPB) void top_quad_kernel(ParentArgs a) {
    constexpr int QUADS = BIG_TPB / 4;
    __shared__ __attribute__((aligned(16))) uint32_t cvs[2][K4T_MAX][8];
    __shared__ __attribute__((aligned(16))) uint32_t msg[QUADS][16];
    // verify: every stored node of the walk fetched up front (one round of
    // loads instead of one dependent global-memory wait per level)
    __shared__ __attribute__((aligned(16))) u32x4 stored[MODE == 1 ? K4T_MAX * 4 : 4];
    const int t = threadIdx.x, q = t & 3, g = t >> 2;
    const uint64_t obj = blockIdx.x;
    uint64_t cnt_prev = a.cnt_prev;
    for (uint64_t i = t; i < cnt_prev; i += BIG_TPB) {
        uint32_t c[8];
        load_cv(a.cv_prev + (obj * a.stride_prev + i) * 32, c);
#pragma unroll
        for (int w = 0; w < 8; ++w) cvs[0][i][w] = c[w];
    }
    if (MODE == 1 && a.stream) {  // level by level: pairs floor(cnt / 2), 16 B per lane of a quad
        const uint8_t *st = a.stream + obj * a.stream_stride;
        uint64_t cnt = cnt_prev, base = 0;
        for (int level = a.level; cnt > 1; ++level) {
            const uint64_t pairs = cnt / 2;
            for (uint64_t i = t; i < 4 * pairs; i += BIG_TPB)
                stored[4 * base + i] = load16_a8(st + parent_stream_off((i >> 2) << level, level, a.N) + 16 * (i & 3));
            base += pairs;
            cnt = (cnt + 1) / 2;
        }
    }
    __syncthreads();
    uint64_t nbase = 0;  // verify: index of this level's first node in `stored`
    const uint32_t slot = (uint32_t)(reinterpret_cast<uintptr_t>(&msg[g][0]) - reinterpret_cast<uintptr_t>(&msg[0][0]));
    const uint8_t *mbase = reinterpret_cast<const uint8_t *>(&msg[0][0]);
    const MsgIdx mi(q, slot);
    const uint32_t iv0 = q == 0 ? IV(0) : q == 1 ? IV(1) : q == 2 ? IV(2) : IV(3);
    const uint32_t iv1 = q == 0 ? IV(4) : q == 1 ? IV(5) : q == 2 ? IV(6) : IV(7);
    bool ok = true;
    int cur = 0;
    for (int level = a.level; cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        for (uint64_t p = g; p < cnt; p += QUADS) {
            if (2 * p + 1 >= cnt_prev) {  // odd last node: promoted unchanged
                cvs[cur ^ 1][p][q] = cvs[cur][2 * p][q];
                cvs[cur ^ 1][p][4 + q] = cvs[cur][2 * p][4 + q];
                continue;
            }
            // message = left CV || right CV: my 16 B are words 4q..4q+3
            const u32x4 mw = *reinterpret_cast<const u32x4 *>(&cvs[cur][2 * p + (q >> 1)][4 * (q & 1)]);
            *reinterpret_cast<u32x4 *>(&msg[g][4 * q]) = mw;
            wave_sync();
            const bool root = cnt == 1;
            uint32_t h0 = iv0, h1 = iv1;
            compress4(h0, h1, mbase, mi, q, iv0, 0, 64, F_PARENT | (root ? F_ROOT : 0u));
            wave_sync();
            if (a.stream) {
                if (MODE == 0) {
                    uint8_t *node = a.stream + obj * a.stream_stride + parent_stream_off(p << level, level, a.N) + 16 * q;
                    store16_a8<false>(node, mw);
                } else {
                    const u32x4 st = stored[4 * (nbase + p) + q];
                    ok &= st.x == mw.x && st.y == mw.y && st.z == mw.z && st.w == mw.w;
                }
            }
            if (root) {
                uint32_t *hp = reinterpret_cast<uint32_t *>(a.hash + obj * 32);
                if (MODE == 0) {
                    hp[q] = h0;
                    hp[4 + q] = h1;
                } else {
                    ok &= hp[q] == h0 && hp[4 + q] == h1;
                }
            } else {
                cvs[cur ^ 1][p][q] = h0;
                cvs[cur ^ 1][p][4 + q] = h1;
            }
        }
        __syncthreads();
        cur ^= 1;
        nbase += cnt_prev / 2;
        cnt_prev = cnt;
    }
    if (MODE == 1 && !ok) flag_mismatch(a.status, obj);
}

}  // namespace small

namespace bao {

bool top_quad_on() {
    static const bool on = [] {
        const char *e = std::getenv("CHIP_TOP_QUAD");
        return !(e && !std::strcmp(e, "0"));
    }();
    return on;
}

hipError_t top_quad_launch(int mode, const ParentArgs &pa, hipStream_t stream) {
    if (pa.cnt_prev > (uint64_t)K4T_MAX || pa.count == 0 || pa.count > 0x7fffffffull) return hipErrorInvalidValue;
    if (mode == 0)
        hipLaunchKernelGGL((small::top_quad_kernel<0>), dim3((unsigned)pa.count), dim3(small::BIG_TPB), 0, stream, pa);
    else
        hipLaunchKernelGGL((small::top_quad_kernel<1>), dim3((unsigned)pa.count), dim3(small::BIG_TPB), 0, stream, pa);
    return hipGetLastError();
}

}  // namespace bao

bool small_ok(uint64_t bao_n, uint64_t count, uint64_t tiny_max) {
    if (!small::enabled() || count == 0) return false;
    const uint64_t N = n_chunks(bao_n);
    return count == 1 ? N <= (uint64_t)KS_MAX_N : N <= tiny_max && count <= 0x7fffffffull;
}

hipError_t small_bao_encode_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                                uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, hipStream_t stream) {
    small::SmallArgs a{};
    a.in = d_in; a.in_stride = in_stride; a.out = d_out; a.out_stride = out_stride;
    a.n = n; a.N = n_chunks(n); a.valid = n; a.count = count;
    a.hash = d_hash;
    return small::launch(0, a, stream);
}

hipError_t small_zfec_bao_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                              uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, hipStream_t stream) {
    if (C == 0 || C % 1024 || !d_out) return hipErrorInvalidValue;
    const void *tab = nullptr;
    hipError_t e = zfec_parity_table(4, 8, &tab);
    if (e != hipSuccess) return e;
    small::SmallArgs a{};
    a.in = d_in; a.in_stride = in_stride; a.out = d_out; a.out_stride = out_stride;
    a.n = 8 * C; a.N = n_chunks(8 * C); a.valid = n; a.C = C; a.count = count;
    a.table = static_cast<const uint32_t *>(tab);
    a.hash = d_hash;
    return small::launch(0, a, stream);
}

hipError_t small_bao_decode_dev(const uint8_t *d_stream, uint64_t in_stride, uint64_t n, uint64_t count,
                                const uint8_t *d_hash, uint8_t *d_out, uint64_t out_stride, uint64_t out_limit,
                                uint32_t *d_status, hipStream_t stream) {
    small::SmallArgs a{};
    a.in = d_stream; a.in_stride = in_stride; a.out = d_out; a.out_stride = out_stride;
    a.n = n; a.N = n_chunks(n); a.out_limit = d_out ? out_limit : 0; a.count = count;
    a.hash = const_cast<uint8_t *>(d_hash);
    a.status = d_status;
    return small::launch(1, a, stream);
}

}  // namespace chip
