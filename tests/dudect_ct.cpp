// dudect_ct.cpp — test infrastructure (tests/test_constant_time.py builds and
// runs it): timing-leak tests of the hand-written constant-time code on the
// secret-key paths, in the style of dudect (Reparaz, Balasch, Verbauwhede,
// "Dude, is my code constant time?", DATE 2017).
//
// Each test times one operation on two classes of secret input — a fixed
// value chosen to stress data-dependent code (1, a low-weight scalar, a
// near-miss tag) and fresh random values — with the class of every
// measurement drawn at random and the measurements interleaved, then runs
// Welch's t-test on the cycle counts (raw, and cropped at the pooled 90th
// and 99th percentile to take out interrupt noise).  A leak shows as a class
// difference: |t| > 4.5.
//   dudect_ct TEST SAMPLES_PER_CLASS      TEST: k1_mul k1_mul_g k1_mul_comb fe_inv sc_sign schnorr_sign gcm_tag all
#include <openssl/crypto.h>
#include <x86intrin.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "../carbonado_amd/csrc/gcm_vaes.hpp"
#include "../carbonado_amd/csrc/secp256k1_host.hpp"
#include "../include/carbonado_hip.h"

// file_container.cpp's file::encode/decode call the device pipeline, which is
// not linked here; these tests never call them.
extern "C" {
uint64_t chip_encode_max_len(uint64_t) { std::abort(); }
int chip_encode(uint8_t, const uint8_t *, uint64_t, const chip_ecies_inject *, const uint8_t *, uint64_t, uint8_t *,
                uint64_t, uint64_t *, uint8_t *, chip_encode_info *) {
    std::abort();
}
int chip_decode(const uint8_t *, uint64_t, const uint8_t *, uint64_t, const uint8_t *, uint64_t, uint32_t, uint8_t,
                uint8_t *, uint64_t, uint64_t *) {
    std::abort();
}
}

namespace k1 = chip::k1;
static std::mt19937_64 rng(0xC0FFEE);
static volatile uint64_t sink;

static void rand_bytes(uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)rng();
}

// a uniformly random scalar in [1, n)
static void rand_scalar(uint8_t k[32]) {
    for (;;) {
        rand_bytes(k, 32);
        const k1::Sc s = k1::sc_from_be(k);
        uint8_t back[32];
        k1::sc_to_be(s, back);
        if (!k1::sc_is_zero(s) && std::memcmp(back, k, 32) == 0) return;  // < n and nonzero
    }
}

struct Welch {
    double n[2] = {0, 0}, mean[2] = {0, 0}, m2[2] = {0, 0};
    void add(int c, double x) {
        n[c] += 1;
        const double d = x - mean[c];
        mean[c] += d / n[c];
        m2[c] += d * (x - mean[c]);
    }
    double t() const {
        const double v0 = m2[0] / (n[0] - 1), v1 = m2[1] / (n[1] - 1);
        return (mean[0] - mean[1]) / std::sqrt(v0 / n[0] + v1 / n[1]);
    }
};

// prep(cls, i) prepares input i of class cls; op(i) runs on it (timed)
static double run(const char *name, size_t per_class, const std::function<void(int, size_t)> &prep,
                  const std::function<void(size_t)> &op) {
    const size_t total = 2 * per_class;
    std::vector<uint8_t> cls(total);
    for (size_t i = 0; i < total; ++i) cls[i] = i < per_class ? 0 : 1;
    std::shuffle(cls.begin(), cls.end(), rng);
    for (size_t i = 0; i < total; ++i) prep(cls[i], i);
    for (size_t i = 0; i < std::min<size_t>(total, 1000); ++i) op(i);  // warm caches and clocks
    std::vector<uint64_t> cyc(total);
    unsigned aux;
    for (size_t i = 0; i < total; ++i) {
        const uint64_t t0 = __rdtscp(&aux);
        op(i);
        const uint64_t t1 = __rdtscp(&aux);
        cyc[i] = t1 - t0;
    }
    std::vector<uint64_t> sorted(cyc);
    std::sort(sorted.begin(), sorted.end());
    const uint64_t p90 = sorted[total * 90 / 100], p99 = sorted[total * 99 / 100];
    Welch raw, c90, c99;
    for (size_t i = 0; i < total; ++i) {
        raw.add(cls[i], (double)cyc[i]);
        if (cyc[i] <= p99) c99.add(cls[i], (double)cyc[i]);
        if (cyc[i] <= p90) c90.add(cls[i], (double)cyc[i]);
    }
    const double worst = std::max({std::fabs(raw.t()), std::fabs(c90.t()), std::fabs(c99.t())});
    std::printf("%-14s n=%zu+%zu median=%llu cyc  t_raw=%+.2f t_p99=%+.2f t_p90=%+.2f  max|t|=%.2f %s\n", name,
                per_class, per_class, (unsigned long long)sorted[total / 2], raw.t(), c99.t(), c90.t(), worst,
                worst < 4.5 ? "PASS" : "LEAK");
    std::fflush(stdout);
    return worst;
}

int main(int argc, char **argv) {
    const std::string which = argc > 1 ? argv[1] : "all";
    const size_t per = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 100000;
    double worst = 0;
    auto want = [&](const char *t) { return which == "all" || which == t; };

    // one affine point P = r G for the k * P tests (public)
    uint8_t r[32], p65[65];
    rand_scalar(r);
    if (!k1::to65(k1::mul_g(r), p65)) return 2;
    const k1::Fe px = k1::fe_from_be(p65 + 1), py = k1::fe_from_be(p65 + 33);
    std::vector<std::array<uint8_t, 32>> in(2 * per);
    uint8_t one[32] = {0};
    one[31] = 1;

    // k * P (ECIES: the receiver's secret on decrypt, the ephemeral on encrypt)
    if (want("k1_mul"))
        worst = std::max(worst, run("k1_mul", per,
            [&](int c, size_t i) { if (c == 0) std::memcpy(in[i].data(), one, 32); else rand_scalar(in[i].data()); },
            [&](size_t i) { sink += k1::mul(in[i].data(), px, py).x.v[0]; }));
    // k * G (ECIES ephemeral key, BIP-340 public key and nonce point)
    if (want("k1_mul_g"))
        worst = std::max(worst, run("k1_mul_g", per,
            [&](int c, size_t i) { if (c == 0) std::memcpy(in[i].data(), one, 32); else rand_scalar(in[i].data()); },
            [&](size_t i) { sink += k1::mul_g(in[i].data()).x.v[0]; }));
    // k * P from a comb table of P (ECIES encrypt for a receiver key seen
    // before: host_stages.cpp peer_mul; the ephemeral scalar is secret)
    if (want("k1_mul_comb")) {
        const k1::CombTable tb(px, py);
        worst = std::max(worst, run("k1_mul_comb", per,
            [&](int c, size_t i) { if (c == 0) std::memcpy(in[i].data(), one, 32); else rand_scalar(in[i].data()); },
            [&](size_t i) { sink += k1::mul_comb(tb, in[i].data()).x.v[0]; }));
    }
    // field inversion (to65: the affine coordinates of a secret-dependent point)
    std::vector<k1::Fe> fe(2 * per);
    if (want("fe_inv"))
        worst = std::max(worst, run("fe_inv", per,
            [&](int c, size_t i) {
                uint8_t b[32];
                if (c == 0) std::memcpy(b, one, 32); else rand_bytes(b, 32);
                b[0] &= 0x7F;  // < p
                fe[i] = k1::fe_from_be(b);
            },
            [&](size_t i) { sink += k1::fe_inv(fe[i]).v[0]; }));
    // the signing scalars: d' = d or n - d, s = k + e d' (mod n)
    uint8_t e32[32];
    rand_bytes(e32, 32);
    const k1::Sc e = k1::sc_from_be(e32);
    const size_t per_sc = std::max<size_t>(per, 1000000);  // ~100 ns each: more samples
    std::vector<std::array<uint8_t, 32>> ds(want("sc_sign") ? 2 * per_sc : 0);
    if (want("sc_sign"))
        worst = std::max(worst, run("sc_sign", per_sc,
            [&](int c, size_t i) { if (c == 0) std::memcpy(ds[i].data(), one, 32); else rand_scalar(ds[i].data()); },
            [&](size_t j) {
                const k1::Sc d = k1::sc_cond_neg(k1::sc_from_be(ds[j].data()), (j & 1) != 0);
                const k1::Sc s = k1::sc_add(k1::sc_from_be(e32), k1::sc_mul(e, d));
                sink += s.v[0];
            }));
    // BIP-340 signing end to end (file.rs:269-271 through file_container.cpp)
    uint8_t msg[32], aux[32];
    rand_bytes(msg, 32);
    rand_bytes(aux, 32);
    if (want("schnorr_sign"))
        worst = std::max(worst, run("schnorr_sign", per,
            [&](int c, size_t i) { if (c == 0) std::memcpy(in[i].data(), one, 32); else rand_scalar(in[i].data()); },
            [&](size_t i) {
                uint8_t sig[64];
                sink += (uint64_t)chip_schnorr_sign(in[i].data(), 32, msg, aux, sig) + sig[63];
            }));
    // the AES-GCM tag check of ECIES decrypt (gcm_vaes.cpp + CRYPTO_memcmp):
    // a tag wrong in its last byte only against a random wrong tag
    uint8_t key[32], iv[16], pt[64], ct[64], tag[16];
    rand_bytes(key, 32);
    rand_bytes(iv, 16);
    rand_bytes(pt, 64);
    {
        chip::host::Gcm g;
        g.init(key, iv, 16, true);
        g.update(pt, 64, ct);
        g.tag(tag);
    }
    std::vector<std::array<uint8_t, 16>> tags(2 * per);
    if (want("gcm_tag") && chip::host::gcm_fast_available())
        worst = std::max(worst, run("gcm_tag", per,
            [&](int c, size_t i) {
                std::memcpy(tags[i].data(), tag, 16);
                if (c == 0) tags[i][15] ^= 1;
                else rand_bytes(tags[i].data(), 16);
            },
            [&](size_t i) {
                chip::host::Gcm g;
                uint8_t out[64], t[16];
                g.init(key, iv, 16, false);
                g.update(ct, 64, out);
                g.tag(t);
                sink += (uint64_t)CRYPTO_memcmp(t, tags[i].data(), 16) + out[0];
                g.wipe();
            }));
    std::printf("max|t| %.2f\n", worst);
    return worst < 4.5 ? 0 : 1;
}
