// api_plans.cpp — zfec encode/decode plans, encode() at Zfec|Bao on the
// device, bao and slice geometry, EncodeInfo, the host-stage glue, and the
// device-side helpers several entry points share.  Shared declarations:
// api_common.hpp.
#include "api_common.hpp"

namespace chip {
namespace api {

bool valid_km(uint32_t k, uint32_t m) { return k >= 1 && m >= k && m <= 256; }

void calc_pad(uint64_t n, uint32_t k, uint32_t *pad, uint64_t *C) {
    const uint64_t unit = 1024ull * k;
    const uint64_t target = (n + unit - 1) / unit * unit;
    *pad = (uint32_t)(target - n);
    *C = target / k;
}

// encode plan: rows 0..k-1 copied, k..m-1 computed from the enc_matrix
// aliased: the data shards already sit in the output (in-place encode), so
// only the m-k parity rows are produced
GfPlan encode_plan(uint32_t k, uint32_t m, uint64_t C, const std::vector<uint8_t> &enc, bool aliased) {
    GfPlan p;
    p.k = k;
    p.np = m - k;
    for (uint32_t j = 0; j < ZF_MAXK; ++j) {
        p.in_off[j] = j < k ? (uint64_t)j * C : 0;
        p.copy_off[j] = (j < k && !aliased) ? (uint64_t)j * C : NO_OUT;
    }
    p.coef.assign(enc.begin() + (size_t)k * k, enc.end());
    for (uint32_t q = 0; q < p.np; ++q) p.comp_off.push_back((uint64_t)(k + q) * C);
    // generic description (output rows as coefficient rows; copies are unit rows)
    p.g_in_off.resize(k);
    for (uint32_t j = 0; j < k; ++j) p.g_in_off[j] = (uint64_t)j * C;
    const uint32_t r0 = aliased ? k : 0;
    for (uint32_t r = r0; r < m; ++r) p.g_out_off.push_back((uint64_t)r * C);
    p.g_coef.assign(enc.begin() + (size_t)r0 * k, enc.end());
    return p;
}

// encode() with Zfec and Bao (encoding.rs:121-147) without the intermediate
// zfec buffer: K1 writes the FEC_M shards of each object straight into their
// chunk slots of the object's bao stream (GfLaunch::bao_off), then K3/K4 hash
// that stream in place (header, parent nodes, hash).  HBM traffic per object:
// n read + m*C written by K1, m*C read + the parents written by K3/K4 (vs an
// extra m*C written and read through a zfec buffer).  C % 1024 == 0 always
// (calc_padding_len pads to a multiple of 1024*k).
//
// K1 is HBM-bound, K3 VALU-bound: a batch is cut into parts and K1 of part
// i+1 runs on one stream beside K3/K4 of part i on another (K1 capped at
// 2 workgroups per CU so K3's waves find room on every CU; 8 parts:
// tools/pipe_sweep.sh, 664 -> 751 GiB/s on 1024 x 16 MiB).
int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

namespace {
struct PipeStreams {  // per thread and device: the two lanes of the overlapped pipeline
    int dev = -1;
    hipStream_t k1 = nullptr, k3 = nullptr;
    hipEvent_t fork = nullptr, k1_done = nullptr, join1 = nullptr, join3 = nullptr;
};
thread_local PipeStreams t_pipe;
hipError_t pipe_streams(PipeStreams **out) {
    PipeStreams &p = t_pipe;
    const int dev = selected_device();
    if (p.dev != dev) {  // first use on this thread, or the process moved to another device
        p = PipeStreams{};
        hipError_t e;
        if ((e = hipStreamCreateWithFlags(&p.k1, hipStreamNonBlocking)) != hipSuccess) return e;
        if ((e = hipStreamCreateWithFlags(&p.k3, hipStreamNonBlocking)) != hipSuccess) return e;
        for (hipEvent_t *ev : {&p.fork, &p.k1_done, &p.join1, &p.join3})
            if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return e;
        p.dev = dev;
    }
    *out = &p;
    return hipSuccess;
}
}  // namespace

// Two stages over `parts` slices of a batch: stage1 (HBM-bound) of part i+1
// runs on one stream beside stage2 (VALU-bound) of part i on another;
// fork/join with events on the caller's stream s.
template <typename S1, typename S2>
hipError_t overlap_parts(uint64_t count, uint64_t parts, hipStream_t s, S1 stage1, S2 stage2) {
    PipeStreams *ps;
    hipError_t e;
    if ((e = pipe_streams(&ps)) != hipSuccess) return e;
    if ((e = hipEventRecord(ps->fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(ps->k1, ps->fork, 0)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(ps->k3, ps->fork, 0)) != hipSuccess) return e;
    for (uint64_t i = 0, o0 = 0; i < parts; ++i) {
        const uint64_t o1 = count * (i + 1) / parts, cnt = o1 - o0;
        if ((e = stage1(o0, cnt, ps->k1)) != hipSuccess) return e;
        if ((e = hipEventRecord(ps->k1_done, ps->k1)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(ps->k3, ps->k1_done, 0)) != hipSuccess) return e;
        if ((e = stage2(o0, cnt, ps->k3)) != hipSuccess) return e;
        o0 = o1;
    }
    if ((e = hipEventRecord(ps->join1, ps->k1)) != hipSuccess) return e;
    if ((e = hipEventRecord(ps->join3, ps->k3)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(s, ps->join1, 0)) != hipSuccess) return e;
    return hipStreamWaitEvent(s, ps->join3, 0);
}


int pipe_parts_cfg() {
    static const int p = env_int("CHIP_PIPE_PARTS", 8);
    return p < 1 ? 1 : p;
}
int pipe_wg_cfg() {
    static const int w = env_int("CHIP_PIPE_K1_WG", 2);
    return w;
}

// K13 (fused_device.hpp) by default: the shards are hashed while they are on
// chip instead of read back from HBM; CHIP_FUSED=0 runs the two-kernel
// overlapped pipeline below (A/B runs).  Scratch: zfec_bao_scratch_len.

// 56 (CHIP_STREAM_OFFSET, read per call so tests can flip it; the caller reads
// it once per batch): every chunk and node of the stream on a 64-B boundary.
// The pipeline line at the level-15 shard length 1002 -> 1110 GiB/s, 16 MiB
// 1091 -> 1132, 1 MiB level-15 shape 982 -> 1077 (profiles/r10i_session).
uint64_t stream_offset() {
    const char *e = std::getenv("CHIP_STREAM_OFFSET");
    const uint64_t o = e ? std::strtoull(e, nullptr, 10) : 56;
    return std::min<uint64_t>(o, 248) & ~(uint64_t)7;
}

bool zfec_bao_any8(uint64_t C, uint64_t count) {
    return fused_on() && !small_ok((uint64_t)CHIP_FEC_M * C, count, KS_TINY_N - 1);
}

hipError_t zfec_bao_dev(const uint8_t *d_in, uint64_t in_stride, uint64_t n, uint64_t count, uint64_t C,
                        uint8_t *d_out, uint64_t out_stride, uint8_t *d_hash, void *d_scratch, hipStream_t s) {
    const uint64_t zlen = (uint64_t)CHIP_FEC_M * C;
    // batches: KS while K13's 8-column blocks are not full (N < 64; r4q: 16 KiB objects 618 vs 393
    // GiB/s, 32 KiB = N 64: K13 737 vs KS 608)
    if (small_ok(zlen, count, KS_TINY_N - 1))
        return small_zfec_bao_dev(d_in, in_stride, n, count, C, d_out, out_stride, d_hash, s);
    if (fused_on()) return zfec_bao_fused_dev(d_in, in_stride, n, count, C, d_out, out_stride, d_hash, d_scratch, s);
    const uint64_t *tab = nullptr;
    hipError_t e = bao_chunk_table(zlen / 1024, &tab);
    if (e != hipSuccess) return e;
    static const std::vector<uint8_t> enc = zfec_enc_matrix(CHIP_FEC_K, CHIP_FEC_M);
    const GfPlan p = encode_plan(CHIP_FEC_K, CHIP_FEC_M, C, enc);
    // parts of at least 64 MiB of shards: smaller batches run the two stages back to back
    const uint64_t parts = std::min<uint64_t>(pipe_parts_cfg(), count * zlen / (64ull << 20));
    if (parts < 2) {
        GfLaunch L{d_in, d_out, in_stride, out_stride, n, C, count};
        L.bao_off = tab;
        e = gf_apply(p, L, s);
        if (e != hipSuccess) return e;
        return bao_encode_inplace_dev(d_out, out_stride, zlen, count, d_hash, d_scratch, s);
    }
    uint8_t *scr = static_cast<uint8_t *>(d_scratch);
    return overlap_parts(
        count, parts, s,
        [&](uint64_t o0, uint64_t cnt, hipStream_t st) {
            GfLaunch L{d_in + o0 * in_stride, d_out + o0 * out_stride, in_stride, out_stride, n, C, cnt};
            L.bao_off = tab;
            L.wg_per_cu = pipe_wg_cfg();
            return gf_apply(p, L, st);
        },
        [&](uint64_t o0, uint64_t cnt, hipStream_t st) {
            hipError_t r = bao_encode_inplace_dev(d_out + o0 * out_stride, out_stride, zlen, cnt, d_hash + 32 * o0,
                                                  scr, st);
            scr += bao_scratch_len(zlen, cnt);
            return r;
        });
}

// decode plan for k selected shares (slot s holds share sel[s], stored at
// in_off[s]); output rows 0..k-1 at r*C
int decode_plan(uint32_t k, uint32_t m, uint64_t C, const std::vector<uint32_t> &sel,
                const std::vector<uint64_t> &slot_off, GfPlan *out) {
    std::vector<uint8_t> enc = zfec_enc_matrix(k, m);
    std::vector<uint8_t> a((size_t)k * k);
    for (uint32_t s = 0; s < k; ++s)
        std::memcpy(&a[(size_t)s * k], &enc[(size_t)sel[s] * k], k);
    if (!gf_invert(a, k)) return CHIP_ERR_ZFEC;
    GfPlan p;
    p.k = k;
    p.np = 0;
    std::vector<int> present(k, -1);
    for (uint32_t s = 0; s < k; ++s)
        if (sel[s] < k) present[sel[s]] = (int)s;
    for (uint32_t j = 0; j < ZF_MAXK; ++j) {
        p.in_off[j] = j < k ? slot_off[j] : 0;
        p.copy_off[j] = NO_OUT;
    }
    p.g_in_off = slot_off;
    for (uint32_t r = 0; r < k; ++r) {
        p.g_out_off.push_back((uint64_t)r * C);
        if (present[r] >= 0) {
            if (k <= ZF_MAXK) p.copy_off[present[r]] = (uint64_t)r * C;
            for (uint32_t s = 0; s < k; ++s) p.g_coef.push_back(s == (uint32_t)present[r] ? 1 : 0);
        } else {
            p.comp_off.push_back((uint64_t)r * C);
            for (uint32_t s = 0; s < k; ++s) p.coef.push_back(a[(size_t)r * k + s]);
            for (uint32_t s = 0; s < k; ++s) p.g_coef.push_back(a[(size_t)r * k + s]);
            p.np++;
        }
    }
    *out = p;
    return CHIP_OK;
}

// choose k distinct shares: primaries first, then secondaries in given order
int select_shares(uint32_t k, uint32_t m, const uint32_t *idx, uint32_t nshares,
                  std::vector<uint32_t> *sel_pos) {
    std::vector<char> have(m, 0);
    sel_pos->clear();
    for (uint32_t s = 0; s < nshares; ++s) {
        if (idx[s] >= m) return CHIP_ERR_ZFEC;
        if (idx[s] < k && !have[idx[s]]) { have[idx[s]] = 1; sel_pos->push_back(s); }
    }
    for (uint32_t s = 0; s < nshares && sel_pos->size() < k; ++s)
        if (idx[s] >= k && !have[idx[s]]) { have[idx[s]] = 1; sel_pos->push_back(s); }
    return sel_pos->size() == k ? CHIP_OK : CHIP_ERR_ZFEC;
}

uint64_t n_chunks_of(uint64_t n) { return n == 0 ? 1 : (n + 1023) / 1024; }

int ceil_log2_u64(uint64_t x) { return x <= 1 ? 0 : 64 - __builtin_clzll(x - 1); }

// chunk range [c0, c1) of a slice request, bao's rules
void slice_chunks(uint64_t n, uint64_t start, uint64_t len, uint64_t *c0, uint64_t *c1) {
    const uint64_t N = n_chunks_of(n);
    uint64_t a = start / 1024;
    if (a >= N) a = N - 1;
    uint64_t end = start + len;  // exclusive byte end
    uint64_t b = end / 1024 + (end % 1024 ? 1 : 0);
    if (b > N) b = N;
    if (b < a + 1) b = a + 1;
    *c0 = a;
    *c1 = b;
}


// pre-order walk of the nodes whose subtree intersects chunks [c0, c1)
void slice_nodes(uint64_t n, uint64_t c0, uint64_t c1, std::vector<SliceNode> *out) {
    const uint64_t N = n_chunks_of(n);
    struct Item { uint64_t s, cnt; };
    std::vector<Item> stack{{0, N}};
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        if (it.s >= c1 || it.s + it.cnt <= c0) continue;
        if (it.cnt == 1) {
            const uint64_t len = (it.s + 1) * 1024 <= n ? 1024 : n - it.s * 1024;
            out->push_back({false, bao_chunk_offset(it.s, N), len, it.s});
            continue;
        }
        const int level = ceil_log2_u64(it.cnt);
        out->push_back({true, bao_parent_offset(it.s, level, N), 64, bao_parent_index(it.s, level, N)});
        const uint64_t left = 1ull << (level - 1);
        stack.push_back({it.s + left, it.cnt - left});  // right after left (LIFO)
        stack.push_back({it.s, left});
    }
}

// EncodeInfo of encode() for format bits Bao|Zfec (encoding.rs:86-172); no device
// EncodeInfo of encode() (encoding.rs:86-171): `input_len` is the caller's
// input, `cur` the length entering zfec (after snap/ecies), bc/be the
// snap/ecies output lengths (0 when the stage is off, encoding.rs:101-115).
int encode_info_for(uint8_t format, uint64_t input_len, uint64_t cur, uint64_t bc, uint64_t be,
                    chip_encode_info *inf, uint64_t *zlen, uint64_t *final_len) {
    std::memset(inf, 0, sizeof *inf);
    inf->input_len = (uint32_t)input_len;  // encoding.rs:87 (as u32)
    inf->bytes_compressed = (uint32_t)bc;
    inf->bytes_encrypted = (uint32_t)be;
    const bool zfec = format & CHIP_FORMAT_ZFEC, bao = format & CHIP_FORMAT_BAO;
    uint64_t cur_len = cur;
    if (zfec) {
        uint32_t pad;
        uint64_t C;
        calc_pad(cur, CHIP_FEC_K, &pad, &C);
        inf->padding_len = pad;
        inf->chunk_len = (uint32_t)C;
        cur_len = (uint64_t)CHIP_FEC_M * C;
        inf->bytes_ecc = (uint32_t)cur_len;                                        // encoding.rs:123
        inf->verifiable_slice_count = (uint16_t)(inf->bytes_ecc / CHIP_SLICE_LEN);  // encoding.rs:124
        if (inf->verifiable_slice_count % 8 != 0) return CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT;
        inf->chunk_slice_count = inf->verifiable_slice_count / 8;                  // encoding.rs:130
    }
    const uint64_t fl = bao ? bao_encoded_len(cur_len) : cur_len;
    if (bao) inf->bytes_verifiable = (uint32_t)fl;
    inf->compression_factor = (float)inf->bytes_compressed / (float)inf->input_len;    // encoding.rs:150
    inf->amplification_factor = (float)inf->bytes_verifiable / (float)inf->input_len;  // encoding.rs:151
    inf->output_len = (uint32_t)fl;
    *zlen = cur_len;
    *final_len = fl;
    return CHIP_OK;
}

bool has_host_stages(uint8_t format) { return format & (CHIP_FORMAT_ECIES | CHIP_FORMAT_SNAPPY); }


// CHIP_STREAM_ENCRYPT=0: snap_compress into a full-size scratch, then
// ecies_encrypt (the two-pass form, for A/B runs)
bool stream_encrypt_on() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_STREAM_ENCRYPT");
        return !(v && v[0] == '0' && v[1] == 0);
    }();
    return on;
}

// bound of the host stages' output for an n-byte input
uint64_t host_stage_max(uint8_t format, uint64_t n) {
    uint64_t m = (format & CHIP_FORMAT_SNAPPY) ? host::snap_max_len(n) : n;
    if (format & CHIP_FORMAT_ECIES) m += host::ECIES_OVERHEAD;
    return m;
}

// snap -> ecies (encoding.rs:101-115) of one object into dst[0..cap); tmp is
// the snap output when both stages run.
int host_stages_into(uint8_t format, const uint8_t *pk, uint64_t pklen, const uint8_t *eph, const uint8_t *nonce,
                     const uint8_t *in, uint64_t n, uint8_t *dst, uint64_t cap, Scratch &tmp,
                     uint64_t *len, uint64_t *bc, uint64_t *be, const host::ChunkSink *sink,
                     uint64_t *filled, const host::EciesKey *prepared, bool par) {
    const bool snap = format & CHIP_FORMAT_SNAPPY, ecies = format & CHIP_FORMAT_ECIES;
    const uint8_t *cur = in;
    uint64_t cur_n = n;
    *bc = *be = 0;
    if (filled) *filled = 0;
    if (ecies && pk && stream_encrypt_on()) {
        // one pass: snappy block -> window -> AES-GCM -> dst (-> stream slots); one
        // object alone (par): its snappy blocks on a few threads
        int st = par && !sink && !prepared
                     ? (snap ? host::ecies_encrypt_par(pk, pklen, eph, nonce, in, n, dst, cap, &cur_n,
                                                       tmp.get(host::SNAP_ECIES_WINDOW))
                             : host::ecies_encrypt_par_plain(pk, pklen, eph, nonce, in, n, dst, cap, &cur_n))
                     : host::ecies_encrypt_stream(pk, pklen, eph, nonce, in, n, snap, dst, cap, &cur_n,
                                                  tmp.get(host::SNAP_ECIES_WINDOW), sink, filled, prepared);
        if (st != CHIP_OK) return st;
        *be = cur_n;
        if (snap) *bc = cur_n - host::ECIES_OVERHEAD;
        *len = cur_n;
        return CHIP_OK;
    }
    if (snap && !ecies && sink && stream_encrypt_on()) {  // frames cut into the stream's chunk slots as they go
        int st = host::snap_compress_stream(in, n, dst, cap, &cur_n, tmp.get(host::SNAP_ECIES_WINDOW), sink, filled);
        if (st != CHIP_OK) return st;
        *bc = *len = cur_n;
        return CHIP_OK;
    }
    if (snap) {
        uint8_t *sd = dst;
        uint64_t scap = cap;
        if (ecies) {
            scap = host::snap_max_len(n) + 1;
            sd = tmp.get(scap);
        }
        // one object alone (par): its blocks on the stage pool's threads
        int st = par ? host::snap_compress_par(in, n, sd, scap, &cur_n) : host::snap_compress(in, n, sd, scap, &cur_n);
        if (st != CHIP_OK) return st;
        cur = sd;
        *bc = cur_n;
    }
    if (ecies) {
        if (!pk) return CHIP_ERR_INVALID_ARG;
        int st = host::ecies_encrypt(pk, pklen, eph, nonce, cur, cur_n, dst, cap, &cur_n);
        if (st != CHIP_OK) return st;
        *be = cur_n;
    }
    *len = cur_n;
    return CHIP_OK;
}

// shares already on the device, contiguous slots of C bytes at d_shares
int zfec_decode_device(uint32_t k, uint32_t m, const uint8_t *d_in, uint64_t in_stride,
                              const std::vector<uint64_t> &slot_off, const std::vector<uint32_t> &sel,
                              uint64_t C, uint64_t count, uint8_t *d_out, uint64_t out_stride,
                              hipStream_t s) {
    GfPlan p;
    int st = decode_plan(k, m, C, sel, slot_off, &p);
    if (st != CHIP_OK) return st;
    GfLaunch L{d_in, d_out, in_stride, out_stride, ~0ull, C, count};
    CHIP_HIP(gf_apply(p, L, s));
    return CHIP_OK;
}

// The content length n of a bao stream of `len` bytes (bao_encoded_len is
// strictly increasing): false when no n gives exactly `len`.
bool bao_content_len(uint64_t len, uint64_t *n) {
    if (len < 8) return false;
    uint64_t lo = 0, hi = len - 8;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (bao_encoded_len(mid) < len) lo = mid + 1;
        else hi = mid;
    }
    *n = lo;
    return bao_encoded_len(lo) == len;
}

// bao-encode `n` device bytes into c->out; hash to host
int bao_encode_ctx(Ctx *c, const uint8_t *d_in, uint64_t n, bool want_stream,
                          uint8_t hash[32]) {
    const uint64_t blen = bao_encoded_len(n);
    if (want_stream) CHIP_HIP(grow(c->out, blen));
    CHIP_HIP(grow(c->scratch, bao_scratch_len(n, 1)));
    CHIP_HIP(grow(c->small, 64));
    uint8_t *d_hash = static_cast<uint8_t *>(c->small.p);
    CHIP_HIP(bao_encode_dev(d_in, 0, n, 1, want_stream ? static_cast<uint8_t *>(c->out.p) : nullptr, 0,
                            d_hash, c->scratch.p, c->stream));
    CHIP_HIP(small_d2h(c, hash, d_hash, 32));
    return CHIP_OK;
}

// verify-decode a device-resident stream of `len` bytes; content -> dst (device)
// `deferred` non-null: the status word lands there at the caller's next
// small_sync (one synchronisation for the verdict and the content copy; the
// caller wipes what it copied out if the verdict is a mismatch)
int bao_decode_ctx(Ctx *c, const uint8_t *d_enc, uint64_t len, uint64_t n, const uint8_t *hash,
                          uint8_t *d_dst, uint64_t out_limit, uint32_t *deferred) {
    (void)len;
    CHIP_HIP(grow(c->scratch, bao_scratch_len(n, 1)));
    CHIP_HIP(grow(c->small, 64));
    uint8_t *d_hash = static_cast<uint8_t *>(c->small.p);
    uint32_t *d_status = reinterpret_cast<uint32_t *>(d_hash + 32);
    uint8_t hs[36] = {};  // the hash and a zero status word, one copy
    std::memcpy(hs, hash, 32);
    CHIP_HIP(small_h2d(c, d_hash, hs, sizeof hs));
    if (out_limit < n)  // only content bytes [0, out_limit) written (every byte verified)
        CHIP_HIP(bao_decode_prefix_dev(d_enc, 0, n, 1, d_hash, d_dst, 0, out_limit, d_status, c->scratch.p,
                                       c->stream));
    else
        CHIP_HIP(bao_decode_dev(d_enc, 0, n, 1, d_hash, d_dst, 0, d_status, c->scratch.p, c->stream));
    if (deferred) {
        *deferred = 0;
        CHIP_HIP(small_d2h(c, deferred, d_status, 4));
        return CHIP_OK;
    }
    uint32_t status = 0;
    CHIP_HIP(small_d2h(c, &status, d_status, 4));
    CHIP_HIP(small_sync(c));
    return status ? (int)status : CHIP_OK;
}

int bao_header(const uint8_t *enc, uint64_t len, uint64_t *n) {
    if (len < 8) return CHIP_ERR_BAO_TRUNCATED;
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)enc[i] << (8 * i);
    // a stream shorter than its header implies is truncated (also guards overflow)
    if (v > len || bao_encoded_len(v) > len) return CHIP_ERR_BAO_TRUNCATED;
    *n = v;
    return CHIP_OK;
}

// node check of one host stream (already H2D'd to c->in); flags to host
int node_check_ctx(Ctx *c, uint64_t n, const uint8_t *hash, std::vector<uint8_t> *cf,
                          std::vector<uint8_t> *pf) {
    const uint64_t N = n_chunks_of(n);
    CHIP_HIP(grow(c->small, 64));
    CHIP_HIP(grow(c->flags, 2 * N + 16));
    uint8_t *d_hash = static_cast<uint8_t *>(c->small.p);
    uint8_t *d_cf = static_cast<uint8_t *>(c->flags.p), *d_pf = d_cf + N;
    CHIP_HIP(small_h2d(c, d_hash, hash, 32));
    CHIP_HIP(bao_node_check(static_cast<const uint8_t *>(c->in.p), 0, n, 1, d_hash, d_cf, d_pf, c->stream));
    cf->resize(N);
    pf->resize(N - 1);
    CHIP_HIP(small_d2h(c, cf->data(), d_cf, N));
    if (N > 1) CHIP_HIP(small_d2h(c, pf->data(), d_pf, N - 1));
    CHIP_HIP(small_sync(c));
    return CHIP_OK;
}

bool slice_ok(uint64_t n, uint64_t c0, uint64_t c1, const std::vector<uint8_t> &cf,
                     const std::vector<uint8_t> &pf) {
    std::vector<SliceNode> nodes;
    slice_nodes(n, c0, c1, &nodes);
    for (const SliceNode &sn : nodes)
        if (!(sn.parent ? pf[sn.index] : cf[sn.index])) return false;
    return true;
}

// scrub()'s repair (decoding.rs:172-209) of one device-resident Bao|Zfec
// stream (content n = 8 C bytes) whose authentic shards are `good`, enqueued
// on the context's stream: zfec decode from them by TRUE index
// (decoding.rs:187), then encode() at Zfec|Bao of the result (the fused
// kernel: shards hashed on chip) into d_dst, its hash to d_h2 (device).  The
// host-side verdicts (too few shares, padding and length mismatch) come back
// at once; the caller compares d_h2 with the expected hash after a sync.  The
// length check is made before the stream is written (the reference makes it
// after encoding; the verdict is the same), so d_dst never receives more
// than `len` bytes.
int scrub_repair_enqueue(Ctx *c, const uint8_t *d_stream, uint64_t n, uint64_t len,
                                const std::vector<uint32_t> &good, uint32_t padding, uint64_t C, uint8_t *d_dst,
                                uint8_t *d_h2) {
    if (good.size() < CHIP_FEC_K) return CHIP_ERR_ZFEC;
    const uint64_t kc = (uint64_t)CHIP_FEC_K * C;
    if (padding > kc) return CHIP_ERR_ZFEC;
    const uint64_t dl = kc - padding;
    uint32_t pad2;
    uint64_t C2;
    calc_pad(dl, CHIP_FEC_K, &pad2, &C2);
    if (pad2 != padding) return CHIP_ERR_SCRUBBED_PADDING_MISMATCH;  // decoding.rs:192-194
    const uint64_t z2 = (uint64_t)CHIP_FEC_M * C2;
    if (bao_encoded_len(z2) != len) return CHIP_ERR_SCRUBBED_LENGTH_MISMATCH;  // decoding.rs:198-203
    std::vector<uint32_t> pos;
    int st = select_shares(CHIP_FEC_K, CHIP_FEC_M, good.data(), (uint32_t)good.size(), &pos);
    if (st != CHIP_OK) return st;
    // content of all shards, parents stripped
    CHIP_HIP(grow(c->mid, n));
    uint8_t *d_z = static_cast<uint8_t *>(c->mid.p);
    CHIP_HIP(bao_gather_content(d_stream, n, 0, n_chunks_of(n), d_z, c->stream));
    std::vector<uint32_t> sel(CHIP_FEC_K);
    std::vector<uint64_t> slot_off(CHIP_FEC_K);
    for (uint32_t s2 = 0; s2 < CHIP_FEC_K; ++s2) { sel[s2] = good[pos[s2]]; slot_off[s2] = sel[s2] * C; }
    CHIP_HIP(grow(c->x1, kc));
    uint8_t *d_dec = static_cast<uint8_t *>(c->x1.p);
    st = zfec_decode_device(CHIP_FEC_K, CHIP_FEC_M, d_z, 0, slot_off, sel, C, 1, d_dec, 0, c->stream);
    if (st != CHIP_OK) return st;
    // re-encode: encoding::zfec then encoding::bao (decoding.rs:191-196), one fused pass
    CHIP_HIP(grow(c->scratch, std::max(zfec_bao_scratch_len(z2, 1), bao_scratch_len(z2, 1))));
    CHIP_HIP(zfec_bao_dev(d_dec, 0, dl, 1, C2, d_dst, 0, d_h2, c->scratch.p, c->stream));
    return CHIP_OK;
}

}  // namespace api
}  // namespace chip
