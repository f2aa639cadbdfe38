// bao_tree.hpp — the bao tree above the chunk CVs (K4 parent levels, the K4t
// top walk, K5b node checks), the K3 launchers (run_bao_t), and the stream
// gathers of extract_slice / verify-decode.  Included at the end of
// bao_device.hpp, whose primitives (b3_parent, node_io, parent_stream_off,
// the K3 chunk body) it builds on.
#pragma once

#include "bao_device.hpp"

namespace chip {
namespace bao {

struct ParentArgs {
    const uint8_t *cv_prev;
    uint8_t *cv_next;
    uint64_t stride_prev, stride_next;  // nodes per object in each buffer
    uint64_t cnt_prev, cnt;             // nodes per object at level-1 and level
    int level;
    uint64_t N, count;
    uint8_t *stream;                    // encode: write parents (may be null); decode: read
    uint64_t stream_stride;
    uint8_t *hash;                      // encode: out; decode: expected
    uint32_t *status;
};

__device__ __forceinline__ void load_cv(const uint8_t *p, uint32_t (&c)[8]) {
    const u32x4 x = reinterpret_cast<const u32x4 *>(p)[0];
    const u32x4 y = reinterpret_cast<const u32x4 *>(p)[1];
    c[0] = x.x; c[1] = x.y; c[2] = x.z; c[3] = x.w; c[4] = y.x; c[5] = y.y; c[6] = y.z; c[7] = y.w;
}

__device__ __forceinline__ void store_cv(uint8_t *p, const uint32_t (&c)[8]) {
    glb(reinterpret_cast<u32x4 *>(p))[0] = u32x4{c[0], c[1], c[2], c[3]};
    glb(reinterpret_cast<u32x4 *>(p))[1] = u32x4{c[4], c[5], c[6], c[7]};
}

// K4: one lane = one node of `level` (parent of two level-1 nodes, or the
// promotion of an odd last node)
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void bao_parent_kernel(ParentArgs a) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.count * a.cnt) return;
    const uint64_t obj = gid / a.cnt;
    const uint64_t q = gid - obj * a.cnt;
    const uint8_t *src = a.cv_prev + (obj * a.stride_prev + 2 * q) * 32;
    uint32_t l[8];
    load_cv(src, l);
    if (2 * q + 1 >= a.cnt_prev) {  // odd last node: promoted unchanged
        store_cv(a.cv_next + (obj * a.stride_next + q) * 32, l);
        return;
    }
    uint32_t r[8], p[8];
    load_cv(src + 32, r);
    const bool root = a.cnt == 1;
    b3_parent(l, r, root, p);
    if (a.stream) {
        uint8_t *node = a.stream + obj * a.stream_stride + parent_stream_off(q << a.level, a.level, a.N);
        if (!node_io<MODE, NT>(node, l, r)) flag_mismatch(a.status, obj);
    }
    if (root) {
        if (MODE == 0) {
            store_cv(a.hash + obj * 32, p);
        } else {
            uint32_t e[8];
            load_cv(a.hash + obj * 32, e);
            bool ok = true;
#pragma unroll
            for (int w = 0; w < 8; ++w) ok &= e[w] == p[w];
            if (!ok) flag_mismatch(a.status, obj);
        }
    } else {
        store_cv(a.cv_next + (obj * a.stride_next + q) * 32, p);
    }
}

// K4t: the top of the tree in one launch.  One workgroup per object walks
// every remaining level (cnt_prev <= K4T_MAX nodes at the first one) with the
// CVs in LDS (2 x cnt_prev x 32 B, dynamic), each level exactly as
// bao_parent_kernel computes it: 13 K4 launches per 16 MiB object become
// 4 + 1.  TPB 64 for batches of many small trees (16384 x 1 MiB objects: one
// wave per object, four times the workgroups per CU of TPB 256, whose waves
// mostly idle above the first level).
constexpr int K4T_MAX = 512;
template <int MODE, bool NT, int TPB = 256>
__global__ __launch_bounds__(TPB) void bao_top_kernel(ParentArgs a) {
    extern __shared__ uint32_t k4t_lds[];
    uint32_t(*cvs[2])[8] = {reinterpret_cast<uint32_t(*)[8]>(k4t_lds),
                            reinterpret_cast<uint32_t(*)[8]>(k4t_lds) + a.cnt_prev};
    const uint64_t obj = blockIdx.x;
    uint64_t cnt_prev = a.cnt_prev;
    for (uint64_t i = threadIdx.x; i < cnt_prev; i += TPB) {
        uint32_t c[8];
        load_cv(a.cv_prev + (obj * a.stride_prev + i) * 32, c);
#pragma unroll
        for (int w = 0; w < 8; ++w) cvs[0][i][w] = c[w];
    }
    __syncthreads();
    int cur = 0;
    bool ok = true;
    for (int level = a.level; cnt_prev > 1; ++level) {
        const uint64_t cnt = (cnt_prev + 1) / 2;
        for (uint64_t q = threadIdx.x; q < cnt; q += TPB) {
            uint32_t l[8], p[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) l[w] = cvs[cur][2 * q][w];
            if (2 * q + 1 >= cnt_prev) {  // odd last node: promoted unchanged
#pragma unroll
                for (int w = 0; w < 8; ++w) cvs[cur ^ 1][q][w] = l[w];
                continue;
            }
            uint32_t r[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) r[w] = cvs[cur][2 * q + 1][w];
            const bool root = cnt == 1;
            b3_parent(l, r, root, p);
            if (a.stream) {
                uint8_t *node = a.stream + obj * a.stream_stride + parent_stream_off(q << level, level, a.N);
                ok &= node_io<MODE, NT>(node, l, r);
            }
            if (root) {
                if (MODE == 0) {
                    store_cv(a.hash + obj * 32, p);
                } else {
                    uint32_t e[8];
                    load_cv(a.hash + obj * 32, e);
#pragma unroll
                    for (int w = 0; w < 8; ++w) ok &= e[w] == p[w];
                }
            } else {
#pragma unroll
                for (int w = 0; w < 8; ++w) cvs[cur ^ 1][q][w] = p[w];
            }
        }
        __syncthreads();
        cur ^= 1;
        cnt_prev = cnt;
    }
    if (!ok) flag_mismatch(a.status, obj);
}

struct CheckArgs {
    const uint8_t *stream;
    uint64_t stream_stride, N, count, nparents;
    const uint8_t *hash;  // expected root hashes [count][32]
    uint8_t *flags;       // [count][nparents], indexed in stream (pre-)order
};

// K5b: every parent node re-hashed from its STORED 64 bytes and compared with
// the copy in its own parent (the root: with the hash).  Independent per node,
// so one launch checks the whole tree; flags are indexed in stream order,
// pidx = P(s) + c(s) - level.
static __global__ __launch_bounds__(256) void bao_parent_check_kernel(CheckArgs a) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= a.count * a.nparents) return;
    const uint64_t obj = gid / a.nparents;
    uint64_t r = gid - obj * a.nparents, cnt = a.N;
    int level = 1;
    for (;; ++level) {  // locate (level, q) of the r-th parent in level order
        const uint64_t np = cnt / 2;
        if (r < np) break;
        r -= np;
        cnt = (cnt + 1) / 2;
    }
    const uint64_t sx = r << level;
    const uint8_t *st = a.stream + obj * a.stream_stride;
    const uint64_t pidx = parents_before(sx, a.N) + parents_at(sx, a.N) - level;
    const uint8_t *node = st + 8 + 1024 * sx + 64 * pidx;
    uint32_t l[8], rr[8], cv[8];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const u32x2 x = reinterpret_cast<const u32x2 *>(node)[w];
        const u32x2 y = reinterpret_cast<const u32x2 *>(node + 32)[w];
        l[2 * w] = x.x; l[2 * w + 1] = x.y; rr[2 * w] = y.x; rr[2 * w + 1] = y.y;
    }
    const bool root = (cnt + 1) / 2 == 1;  // this level has a single node
    b3_parent(l, rr, root, cv);
    bool ok;
    if (root) {
        ok = true;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t e = (uint32_t)a.hash[obj * 32 + 4 * w] | (uint32_t)a.hash[obj * 32 + 4 * w + 1] << 8 |
                               (uint32_t)a.hash[obj * 32 + 4 * w + 2] << 16 |
                               (uint32_t)a.hash[obj * 32 + 4 * w + 3] << 24;
            ok &= e == cv[w];
        }
    } else {
        ok = stored_slot_matches(st, sx, level, a.N, cv);
    }
    a.flags[obj * a.nparents + pidx] = ok ? 1 : 0;
}

__host__ __device__ inline uint64_t n_chunks(uint64_t n) { return n == 0 ? 1 : (n + 1023) / 1024; }

template <int CPL>
inline uint64_t bao_scratch_len_t(uint64_t n, uint64_t count) {
    const uint64_t N0 = (n_chunks(n) + CPL - 1) / CPL;
    return count * 32 * (N0 + (N0 + 1) / 2);
}

// K4t with a quad (four lanes) per parent for up to TOP_QUAD_MAX objects,
// whose tree top is latency-bound (small_kernels.hip; CHIP_TOP_QUAD=0: off)
constexpr uint64_t TOP_QUAD_MAX = 8;
bool top_quad_on();
hipError_t top_quad_launch(int mode, const ParentArgs &pa, hipStream_t stream);

// The tree above a level of node CVs: K4 per level, then K4t for the top
// once a level has <= K4T_MAX nodes.  cv_prev [count][stride_prev] holds the
// cnt_prev nodes of level `level - 1`; cv_next (stride_next >= ceil(cnt_prev/2))
// is the ping-pong buffer.  Parents are written into (MODE 0) or checked
// against (MODE 1) the streams, the root into / against d_hash.
template <int MODE, bool BAO_NTS>
hipError_t run_parent_levels(uint8_t *cv_prev, uint64_t stride_prev, uint64_t cnt_prev, int level, uint8_t *cv_next,
                             uint64_t stride_next, uint64_t N, uint64_t count, uint8_t *stream_buf, uint64_t sstride,
                             uint8_t *d_hash, uint32_t *d_status, hipStream_t stream) {
    uint8_t *prev = cv_prev, *next = cv_next;
    uint64_t sp = stride_prev, sn = stride_next;
    for (; cnt_prev > 1; ++level) {
        ParentArgs pa;
        pa.cv_prev = prev; pa.cv_next = next; pa.stride_prev = sp; pa.stride_next = sn;
        pa.cnt_prev = cnt_prev; pa.cnt = (cnt_prev + 1) / 2; pa.level = level;
        pa.N = N; pa.count = count; pa.stream = stream_buf; pa.stream_stride = sstride;
        pa.hash = d_hash; pa.status = d_status;
        if (cnt_prev <= (uint64_t)K4T_MAX && count <= 0x7fffffffull) {  // the rest of the tree, one launch
            if (count <= TOP_QUAD_MAX && top_quad_on()) return top_quad_launch(MODE, pa, stream);
            const size_t lds = 2 * cnt_prev * 32;
            if (count >= 2048)
                hipLaunchKernelGGL((bao_top_kernel<MODE, BAO_NTS, 64>), dim3((unsigned)count), dim3(64), lds, stream,
                                   pa);
            else
                hipLaunchKernelGGL((bao_top_kernel<MODE, BAO_NTS>), dim3((unsigned)count), dim3(256), lds, stream, pa);
            return hipGetLastError();
        }
        const uint64_t work = count * pa.cnt;
        hipLaunchKernelGGL((bao_parent_kernel<MODE, BAO_NTS>), dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                           stream, pa);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        cnt_prev = pa.cnt;
        std::swap(prev, next);
        std::swap(sp, sn);
    }
    return hipSuccess;
}

// The K3 kernel of a configuration: ChunkKernel<...>::fn.  The library
// (bao_kernels.hip) specialises it for the configurations it ships, each a
// kernel of its own name (bao_chunk_kernel_encode, _verify, _check,
// _inplace, and their _static forms without the run queue);
// tools/bao_variants.hpp defines it for every configuration.
template <int MODE, int CPL, bool NTS, int SP, int SU, int SE, int XG, bool DQ>
struct ChunkKernel;

// Enqueue K3 over `waves` wave tasks: with DQ a persistent grid of resident
// workgroups taking wave tasks from the stream's run queue, else one wave per
// task.
template <int MODE, int CPL, bool NTS, int SP, int SU, int SE, int XG, bool DQ>
hipError_t launch_chunk_kernel(ChunkArgs ca, hipStream_t stream, size_t pad_lds) {
    const uint64_t waves = ca.count * ((ca.N + 64ull * CPL - 1) / (64ull * CPL));
    const uint64_t blocks = (waves + K3_WAVES - 1) / K3_WAVES;
    bool dq = DQ && waves < (1ull << 31);
    if (dq) {  // persistent grid of resident workgroups, wave tasks from the stream's run queue
        uint32_t *q = nullptr;
        const void *fn = reinterpret_cast<const void *>(ChunkKernel<MODE, CPL, NTS, SP, SU, SE, XG, true>::fn);
        // per instance and LDS pad, asked once: the query costs ~6 us of API
        // time, which single small objects paid on every call (profiles/r4c)
        static std::mutex occ_mu;
        static std::map<size_t, int> occ;
        int per_cu = 0;
        {
            std::lock_guard<std::mutex> lk(occ_mu);
            auto it = occ.find(pad_lds);
            if (it != occ.end()) {
                per_cu = it->second;
            } else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, K3_TPB, pad_lds) == hipSuccess) {
                occ[pad_lds] = per_cu;
            } else {
                per_cu = 0;
            }
        }
        dq = per_cu > 0 && stream_queue(stream, &q) == hipSuccess;
        (void)hipGetLastError();
        if (dq) {
            ca.queue = q + QUEUE_K3;
            const uint64_t grid = std::min<uint64_t>(blocks, (uint64_t)per_cu * (uint64_t)num_cus());
            hipLaunchKernelGGL((ChunkKernel<MODE, CPL, NTS, SP, SU, SE, XG, true>::fn), dim3((unsigned)grid),
                               dim3(K3_TPB), pad_lds, stream, ca);
        }
    }
    if (!dq)
        hipLaunchKernelGGL((ChunkKernel<MODE, CPL, NTS, SP, SU, SE, XG, false>::fn), dim3((unsigned)blocks),
                           dim3(K3_TPB), pad_lds, stream, ca);
    return hipGetLastError();
}

// Enqueue K3 then one K4 launch per remaining level.
template <int MODE, int BAO_CPL, bool BAO_NTS, int SP = 0, int SU = 1, int SE = 0, int XG = 0, bool DQ = false>
hipError_t run_bao_t(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count,
                   uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, uint32_t *d_status,
                   void *d_scratch, hipStream_t stream, size_t pad_lds = 0 /* tuning: occupancy probe */,
                   uint64_t out_limit = ~0ull /* decode: content prefix written */) {
    if (count == 0) return hipSuccess;
    const uint64_t N = n_chunks(n);
    constexpr int LOG = ilog2(BAO_CPL);
    const uint64_t N0 = (N + BAO_CPL - 1) / BAO_CPL;  // nodes at level LOG
    uint8_t *bufA = static_cast<uint8_t *>(d_scratch);
    uint8_t *bufB = bufA + count * N0 * 32;
    const uint64_t strideA = N0, strideB = (N0 + 1) / 2;

    ChunkArgs ca;
    ca.in = d_in; ca.out = d_out; ca.in_stride = in_stride; ca.out_stride = out_stride;
    ca.n = n; ca.N = N; ca.count = count; ca.cv = bufA; ca.cv_stride = strideA;
    ca.hash = d_hash; ca.status = d_status;
    ca.out_limit = out_limit;
    hipError_t e = launch_chunk_kernel<MODE, BAO_CPL, BAO_NTS, SP, SU, SE, XG, DQ>(ca, stream, pad_lds);
    if (e != hipSuccess) return e;

    uint8_t *stream_buf = (MODE == 0 || MODE == 3) ? d_out : const_cast<uint8_t *>(d_in);
    const uint64_t sstride = (MODE == 0 || MODE == 3) ? out_stride : in_stride;
    return run_parent_levels<MODE == 3 ? 0 : MODE, BAO_NTS>(bufA, strideA, N0, LOG + 1, bufB, strideB, N, count,
                                                           stream_buf, sstride, d_hash, d_status, stream);
}

// Gather the content of chunks [c0, c1) of one stream into a contiguous buffer
// (the inverse of the layout: strips the interleaved parent nodes).
static __global__ __launch_bounds__(256) void bao_gather_kernel(const uint8_t *stream, uint64_t n, uint64_t N,
                                                         uint64_t c0, uint64_t c1, uint8_t *out) {
    const uint64_t bytes = (c1 * 1024 < n ? c1 * 1024 : n) - c0 * 1024;
    for (uint64_t b = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; b < bytes;
         b += (uint64_t)gridDim.x * 256 * 16) {
        const uint64_t ci = c0 + b / 1024;
        const uint8_t *src = stream + chunk_stream_off(ci, N) + (b % 1024);
        if (b + 16 <= bytes) {
            *reinterpret_cast<u32x4 *>(out + b) = load16_a8(src);
        } else {
            for (uint64_t q = 0; b + q < bytes; ++q) out[b + q] = src[q];
        }
    }
}

// The parent nodes in front of chunks [0, nd) of `count` streams (N chunks,
// coff = bao_chunk_table(N)), in stream order, to nodes + o * nodes_stride.
// encode() from host memory at Zfec|Bao: chunks [0, nd) are the data shards,
// which the host already holds, so only these nodes and the stream's tail
// cross PCIe (api_encode.cpp SplitGeo).  Lane = 8 B of one run of nodes; the
// runs sit at 8 mod 64, so 8-B accesses.
static __global__ __launch_bounds__(256) void bao_data_nodes_kernel(const uint8_t *stream, uint64_t stride,
                                                                    const uint64_t *coff, uint64_t nd,
                                                                    uint64_t count, uint8_t *nodes,
                                                                    uint64_t nodes_stride) {
    const uint64_t per = nd * 8, total = count * per;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
        const uint64_t o = t / per, r = t % per, i = r / 8, q = r % 8;
        const uint64_t end = coff[i], beg = i ? coff[i - 1] + 1024 : 8;
        const uint64_t before = (beg - 8 - 1024 * i) / 64;  // data-region nodes ahead of this run
        const uint8_t *s = stream + o * stride + beg + 8 * q;
        uint8_t *d = nodes + o * nodes_stride + 64 * before + 8 * q;
        for (uint64_t b = 0; b < end - beg; b += 64)
            *reinterpret_cast<uint64_t *>(d + b) = *reinterpret_cast<const uint64_t *>(s + b);
    }
}

// Content bytes [0, nbytes) of `count` streams (chunk i at coff[i] of each
// row) to contiguous rows: encode() from host memory at Ecies|Zfec|Bao,
// whose host stage wrote the zfec input straight into the stream's chunk
// slots.  Lane = 8 B (the slots sit at 8 mod 64).
static __global__ __launch_bounds__(256) void bao_gather_rows_kernel(const uint8_t *stream, uint64_t stride,
                                                                     const uint64_t *coff, uint64_t count,
                                                                     uint64_t nbytes, uint8_t *out,
                                                                     uint64_t out_stride) {
    const uint64_t words = (nbytes + 7) / 8, total = count * words;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
        const uint64_t o = t / words, b = 8 * (t % words);
        const uint8_t *s = stream + o * stride + coff[b / 1024] + b % 1024;
        uint8_t *d = out + o * out_stride + b;
        if (b + 8 <= nbytes) {
            *reinterpret_cast<uint64_t *>(d) = *reinterpret_cast<const uint64_t *>(s);
        } else {
            for (uint64_t q = 0; b + q < nbytes; ++q) d[q] = s[q];
        }
    }
}

// Per-node verification flags of `count` streams of content length n:
// chunk_flags [count][N], parent_flags [count][N-1] (stream order).
template <int BAO_NTS_UNUSED = 0>
hipError_t run_node_check(const uint8_t *d_stream, uint64_t stride, uint64_t n, uint64_t count,
                          const uint8_t *d_hash, uint8_t *chunk_flags, uint8_t *parent_flags, hipStream_t stream) {
    const uint64_t N = n_chunks(n);
    ChunkArgs ca;
    ca.in = d_stream; ca.out = nullptr; ca.in_stride = stride; ca.out_stride = 0;
    ca.n = n; ca.N = N; ca.count = count; ca.cv = chunk_flags; ca.cv_stride = N;
    ca.hash = const_cast<uint8_t *>(d_hash); ca.status = nullptr;
    // persistent grid, wave tasks from the run queue (as decode); scrub's batch check
    hipError_t e = launch_chunk_kernel<2, 1, false, 0, 1, 0, 1, true>(ca, stream, 0);
    if (e != hipSuccess || N < 2) return e;
    CheckArgs pa{d_stream, stride, N, count, N - 1, d_hash, parent_flags};
    const uint64_t work = count * (N - 1);
    hipLaunchKernelGGL(bao_parent_check_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, pa);
    return hipGetLastError();
}

}  // namespace bao
}  // namespace chip
