// abi_latency.cpp — single-object encode()/decode() latency through the C-ABI,
// three ways per row:
//   lib    chip_encode / chip_decode, the caller's buffers allocated once and
//          reused (a service encoding segment after segment);
//   patch  the call sequence carbonado-hip/reroute.patch makes under the `hip`
//          feature, each output a fresh allocation as the Rust wrappers'
//          Vec::with_capacity (lib.rs into_vec): Zfec|Bao one chip_encode /
//          chip_decode (format 12), Zfec or Bao alone the stage call; at levels
//          with Snappy/Ecies the host crates run first (in Rust under the patch;
//          here chip_snap_compress / chip_ecies_encrypt stand in for them);
//   r5     round 5's patch at Zfec|Bao: chip_zfec_encode -> host Vec ->
//          chip_bao_encode, and chip_bao_decode -> host Vec -> chip_zfec_decode.
// The three are interleaved per repetition (same box state); medians.
//   g++ -std=c++17 -O2 tools/abi_latency.cpp -Iinclude -Lcarbonado_amd/lib -lcarbonado_hip
//       -Wl,-rpath,'$ORIGIN/../carbonado_amd/lib' -o tools/abi_latency
//   abi_latency [REPS] [LEVELS, e.g. 12,4,8] [SIZES in bytes, e.g. 1024,1048576]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../include/carbonado_hip.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ABI_LAT_STAGES=1: each patch-sequence step's time to stderr (us)
static void stage_mark(const char *what, double *t) {
    static const bool on = [] {
        const char *v = std::getenv("ABI_LAT_STAGES");
        return v && v[0] == '1';
    }();
    if (!on) return;
    const double n = now_us();
    std::fprintf(stderr, "[patch] %-14s %8.1f us\n", what, n - *t);
    *t = n;
}

static std::vector<uint64_t> parse_list(const char *s, std::vector<uint64_t> def) {
    if (!s) return def;
    std::vector<uint64_t> v;
    std::stringstream ss(s);
    std::string t;
    while (std::getline(ss, t, ',')) v.push_back(std::strtoull(t.c_str(), nullptr, 10));
    return v;
}

static double median(std::vector<double> v) {
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    return v[v.size() / 2];
}

// a Rust Vec::with_capacity: malloc'd, uninitialised, freed after use
struct Fresh {
    uint8_t *p;
    explicit Fresh(uint64_t n) : p(static_cast<uint8_t *>(std::malloc(n ? n : 1))) {}
    ~Fresh() { std::free(p); }
};

struct Obj {
    int level;
    std::vector<uint8_t> in;
    const uint8_t *pub, *sk;
    chip_ecies_inject inj;
};

// encoding::encode under the patch; returns the status, the stream's length in *elen
static int patch_encode(const Obj &o, std::vector<uint8_t> *keep, uint8_t hash[32], chip_encode_info *info) {
    const uint8_t *cur = o.in.data();
    uint64_t cur_n = o.in.size();
    double t = now_us();
    Fresh snap(o.level & CHIP_FORMAT_SNAPPY ? chip_snap_max_len(cur_n) : 0);
    if (o.level & CHIP_FORMAT_SNAPPY) {
        uint64_t l = 0;
        if (int st = chip_snap_compress(cur, cur_n, snap.p, chip_snap_max_len(cur_n), &l)) return st;
        stage_mark("enc snap", &t);
        cur = snap.p;
        cur_n = l;
    }
    Fresh ecies(o.level & CHIP_FORMAT_ECIES ? cur_n + 97 : 0);
    if (o.level & CHIP_FORMAT_ECIES) {
        uint64_t l = 0;
        if (int st = chip_ecies_encrypt(o.pub, 65, &o.inj, cur, cur_n, ecies.p, cur_n + 97, &l)) return st;
        stage_mark("enc ecies", &t);
        cur = ecies.p;
        cur_n = l;
    }
    const int zb = o.level & (CHIP_FORMAT_ZFEC | CHIP_FORMAT_BAO);
    uint64_t len = 0;
    int st = CHIP_OK;
    if (zb == (CHIP_FORMAT_ZFEC | CHIP_FORMAT_BAO)) {
        const uint64_t cap = chip_encode_max_len(cur_n);
        Fresh out(cap);
        st = chip_encode(12, nullptr, 0, nullptr, cur, cur_n, out.p, cap, &len, hash, info);
        if (st == CHIP_OK && keep) keep->assign(out.p, out.p + len);
    } else if (zb == CHIP_FORMAT_ZFEC) {
        const uint64_t cap = chip_zfec_encoded_len(cur_n, 4, 8);
        Fresh out(cap);
        uint32_t pad = 0, chunk = 0;
        st = chip_zfec_encode(4, 8, cur, cur_n, out.p, cap, &pad, &chunk);
        info->padding_len = pad;
        if (st == CHIP_OK && keep) keep->assign(out.p, out.p + cap);
    } else if (zb == CHIP_FORMAT_BAO) {
        const uint64_t cap = chip_bao_encoded_len(cur_n);
        Fresh out(cap);
        st = chip_bao_encode(cur, cur_n, out.p, cap, &len, hash);
        if (st == CHIP_OK && keep) keep->assign(out.p, out.p + len);
    }
    stage_mark("enc zfec/bao", &t);
    return st;
}

// decoding::decode under the patch
static int patch_decode(const Obj &o, const std::vector<uint8_t> &enc, const uint8_t hash[32], uint32_t padding,
                        std::vector<uint8_t> *keep) {
    const int zb = o.level & (CHIP_FORMAT_ZFEC | CHIP_FORMAT_BAO);
    const uint8_t *cur = enc.data();
    uint64_t cur_n = enc.size(), len = 0;
    double t = now_us();
    Fresh dev(std::max<uint64_t>(cur_n, 1024));
    int st = CHIP_OK;
    if (zb == (CHIP_FORMAT_ZFEC | CHIP_FORMAT_BAO)) {
        st = chip_decode(nullptr, 0, hash, 32, cur, cur_n, padding, 12, dev.p, std::max<uint64_t>(cur_n, 1024), &len);
    } else if (zb == CHIP_FORMAT_ZFEC) {
        st = chip_zfec_decode(4, 8, cur, cur_n, padding, dev.p, cur_n / 8 * 4, &len);
    } else if (zb == CHIP_FORMAT_BAO) {
        st = chip_bao_decode(cur, cur_n, hash, 32, dev.p, cur_n, &len);
    }
    if (st) return st;
    stage_mark("dec zfec/bao", &t);
    cur = dev.p;
    cur_n = len;
    Fresh dec(o.level & CHIP_FORMAT_ECIES ? cur_n : 0);
    if (o.level & CHIP_FORMAT_ECIES) {
        if ((st = chip_ecies_decrypt(o.sk, 32, cur, cur_n, dec.p, cur_n, &len))) return st;
        stage_mark("dec ecies", &t);
        cur = dec.p;
        cur_n = len;
    }
    const uint64_t ucap = o.in.size() + 1024;
    Fresh un(o.level & CHIP_FORMAT_SNAPPY ? ucap : 0);
    if (o.level & CHIP_FORMAT_SNAPPY) {
        if ((st = chip_snap_decompress(cur, cur_n, un.p, ucap, &len))) return st;
        stage_mark("dec snap", &t);
        cur = un.p;
        cur_n = len;
    }
    if (keep) keep->assign(cur, cur + cur_n);
    return CHIP_OK;
}

// round 5's patch at Zfec|Bao: two stage calls, a host Vec between them
static int r5_encode(const Obj &o, std::vector<uint8_t> *keep, uint8_t hash[32]) {
    const uint64_t n = o.in.size(), zcap = chip_zfec_encoded_len(n, 4, 8);
    Fresh z(zcap);
    uint32_t pad = 0, chunk = 0;
    if (int st = chip_zfec_encode(4, 8, o.in.data(), n, z.p, zcap, &pad, &chunk)) return st;
    const uint64_t bcap = chip_bao_encoded_len(zcap);
    Fresh b(bcap);
    uint64_t len = 0;
    if (int st = chip_bao_encode(z.p, zcap, b.p, bcap, &len, hash)) return st;
    if (keep) keep->assign(b.p, b.p + len);
    return CHIP_OK;
}

static int r5_decode(const std::vector<uint8_t> &enc, const uint8_t hash[32], uint32_t padding,
                     std::vector<uint8_t> *keep) {
    Fresh v(enc.size());
    uint64_t vl = 0, len = 0;
    if (int st = chip_bao_decode(enc.data(), enc.size(), hash, 32, v.p, enc.size(), &vl)) return st;
    Fresh d(vl / 8 * 4 + 1);
    if (int st = chip_zfec_decode(4, 8, v.p, vl, padding, d.p, vl / 8 * 4, &len)) return st;
    if (keep) keep->assign(d.p, d.p + len);
    return CHIP_OK;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 50;
    const auto levels = parse_list(argc > 2 ? argv[2] : nullptr, {12, 4, 8, 15});
    const auto sizes = parse_list(argc > 3 ? argv[3] : nullptr, {1024, 65536, 1 << 20, 4 << 20, 16 << 20});
    uint8_t sk[32], pub[65], eph[32], nonce[16];
    std::mt19937_64 rng(7);
    for (auto &x : sk) x = (uint8_t)rng();
    for (auto &x : eph) x = (uint8_t)rng();
    for (auto &x : nonce) x = (uint8_t)rng();
    sk[0] &= 0x7f;
    eph[0] &= 0x7f;
    if (chip_ecies_public_key(sk, pub) != CHIP_OK) return 1;
    std::printf("%5s %9s %9s %9s %9s %9s %9s %9s  (median us of %d, interleaved)\n", "level", "bytes", "lib_enc",
                "lib_dec", "patch_enc", "patch_dec", "r5_enc", "r5_dec", reps);
    for (uint64_t level : levels) {
        for (uint64_t n : sizes) {
            Obj o{(int)level, std::vector<uint8_t>(n), pub, sk, {eph, nonce}};
            for (auto &x : o.in) x = (uint8_t)rng();
            if (const char *dk = std::getenv("ABI_LAT_DATA"); dk && !std::strcmp(dk, "text")) {
                // compressible input for the snappy stage: words from a small vocabulary
                static const char *words[] = {"carbonado ", "apocalypse ", "resistant ", "storage ", "segment ",
                                              "zfec ", "bao ", "stream ", "verifiable ", "encode ", "0x3f, ",
                                              "{\"id\": ", "\n", "return ", "hash(", ") "};
                for (size_t p = 0; p < n;) {
                    const char *w = words[rng() % 16];
                    for (size_t k = 0; w[k] && p < n; ++k) o.in[p++] = (uint8_t)w[k];
                }
            }
            std::vector<uint8_t> enc(chip_encode_max_len(n)), dec(n + (n >> 3) + 4096);
            uint8_t hash[32], hp[32], h5[32];
            chip_encode_info info{}, pinfo{};
            uint64_t elen = 0, dlen = 0;
            auto lib_enc = [&] {
                return chip_encode((uint8_t)level, pub, 65, &o.inj, o.in.data(), n, enc.data(), enc.size(), &elen,
                                   hash, &info);
            };
            auto lib_dec = [&] {
                return chip_decode(sk, 32, hash, 32, enc.data(), elen, info.padding_len, (uint8_t)level, dec.data(),
                                   dec.size(), &dlen);
            };
            // correctness of all three before timing: same stream, same content back
            std::vector<uint8_t> penc, pdec, renc, rdec;
            const bool zb = (level & 12) == 12;
            if (lib_enc() != CHIP_OK || lib_dec() != CHIP_OK || dlen != n ||
                !std::equal(o.in.begin(), o.in.end(), dec.begin()) || patch_encode(o, &penc, hp, &pinfo) != CHIP_OK ||
                penc.size() != elen || std::memcmp(penc.data(), enc.data(), elen) ||
                patch_decode(o, penc, hp, pinfo.padding_len, &pdec) != CHIP_OK || pdec != o.in ||
                (zb && !(level & 3) &&
                 (r5_encode(o, &renc, h5) != CHIP_OK || renc != penc || std::memcmp(h5, hp, 32) ||
                  r5_decode(renc, h5, pinfo.padding_len, &rdec) != CHIP_OK || rdec != o.in))) {
                std::printf("level %llu n %llu: round trip or stream mismatch\n", (unsigned long long)level,
                            (unsigned long long)n);
                return 1;
            }
            const int r = std::max(3, n >= (16u << 20) ? reps / 3 : reps);
            std::vector<double> te, td, pe, pd, re, rd;
            for (int i = 0; i < r; ++i) {
                double t = now_us();
                lib_enc();
                te.push_back(now_us() - t);
                t = now_us();
                lib_dec();
                td.push_back(now_us() - t);
                t = now_us();
                patch_encode(o, nullptr, hp, &pinfo);
                pe.push_back(now_us() - t);
                t = now_us();
                patch_decode(o, penc, hp, pinfo.padding_len, nullptr);
                pd.push_back(now_us() - t);
                if (zb && !(level & 3)) {
                    t = now_us();
                    r5_encode(o, nullptr, h5);
                    re.push_back(now_us() - t);
                    t = now_us();
                    r5_decode(renc, h5, pinfo.padding_len, nullptr);
                    rd.push_back(now_us() - t);
                }
            }
            std::printf("%5llu %9llu %9.1f %9.1f %9.1f %9.1f", (unsigned long long)level, (unsigned long long)n,
                        median(te), median(td), median(pe), median(pd));
            if (!re.empty()) std::printf(" %9.1f %9.1f\n", median(re), median(rd));
            else std::printf(" %9s %9s\n", "-", "-");
            std::fflush(stdout);
        }
    }
    return 0;
}
