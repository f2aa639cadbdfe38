// scrub_latency.cpp — one call's latency of the rerouted scrub / verify_slice /
// extract_slice (decoding.rs:116-212) through the C-ABI, for a clean level-12
// stream (scrub answers UnnecessaryScrub) and one with a flipped byte
// (scrub repairs it), median us of REPS.
//   g++ -std=c++17 -O2 tools/scrub_latency.cpp -Iinclude -Lcarbonado_amd/lib -lcarbonado_hip
//       -Wl,-rpath,'$ORIGIN/../carbonado_amd/lib' -o tools/scrub_latency
//   scrub_latency [REPS] [SIZES in bytes]
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

template <class F>
static double median_us(int reps, F f) {
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const double a = now_us();
        f();
        t.push_back(now_us() - a);
    }
    std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 30;
    std::vector<uint64_t> sizes{65536, 1 << 20, 4 << 20, 16 << 20};
    if (argc > 2) {
        sizes.clear();
        std::stringstream ss(argv[2]);
        std::string t;
        while (std::getline(ss, t, ',')) sizes.push_back(std::strtoull(t.c_str(), nullptr, 10));
    }
    std::printf("%9s %11s %11s %11s %11s %11s  (median us of %d; level 12)\n", "bytes", "scrub_ok", "scrub_fix",
                "verify_1", "verify_mid", "extract", reps);
    std::mt19937_64 rng(5);
    for (uint64_t n : sizes) {
        std::vector<uint8_t> in(n);
        for (auto &x : in) x = (uint8_t)rng();
        std::vector<uint8_t> enc(chip_encode_max_len(n)), out(enc.size() + 4096), bad;
        uint64_t elen = 0, olen = 0;
        uint8_t hash[32];
        chip_encode_info info{};
        if (chip_encode(12, nullptr, 0, nullptr, in.data(), n, enc.data(), enc.size(), &elen, hash, &info) != CHIP_OK)
            return 1;
        enc.resize(elen);
        bad = enc;
        bad[elen / 3] ^= 0x20;
        // the verdicts first: clean -> UnnecessaryScrub, damaged -> the clean stream back
        if (chip_scrub(enc.data(), elen, hash, 32, info.padding_len, info.chunk_len, out.data(), out.size(), &olen) !=
            CHIP_ERR_UNNECESSARY_SCRUB) {
            std::printf("n %llu: clean scrub verdict\n", (unsigned long long)n);
            return 1;
        }
        if (chip_scrub(bad.data(), elen, hash, 32, info.padding_len, info.chunk_len, out.data(), out.size(), &olen) !=
                CHIP_OK ||
            olen != elen || std::memcmp(out.data(), enc.data(), elen)) {
            std::printf("n %llu: repair\n", (unsigned long long)n);
            return 1;
        }
        const uint64_t mid = (n / 1024) / 2;
        if (chip_bao_verify_slice(hash, 32, enc.data(), elen, mid, 1, out.data(), out.size(), &olen) != CHIP_OK ||
            olen != std::min<uint64_t>(1024, n - mid * 1024)) {
            std::printf("n %llu: verify_slice\n", (unsigned long long)n);
            return 1;
        }
        const double s_ok = median_us(reps, [&] {
            chip_scrub(enc.data(), elen, hash, 32, info.padding_len, info.chunk_len, out.data(), out.size(), &olen);
        });
        const double s_fix = median_us(reps, [&] {
            chip_scrub(bad.data(), elen, hash, 32, info.padding_len, info.chunk_len, out.data(), out.size(), &olen);
        });
        const double v1 = median_us(reps, [&] {
            chip_bao_verify_slice(hash, 32, enc.data(), elen, 0, 1, out.data(), out.size(), &olen);
        });
        const double vm = median_us(reps, [&] {
            chip_bao_verify_slice(hash, 32, enc.data(), elen, mid, 1, out.data(), out.size(), &olen);
        });
        const double ex = median_us(reps, [&] {
            chip_bao_extract_slice(enc.data(), elen, mid, 1024, out.data(), out.size(), &olen);
        });
        std::printf("%9llu %11.1f %11.1f %11.1f %11.1f %11.1f\n", (unsigned long long)n, s_ok, s_fix, v1, vm, ex);
        std::fflush(stdout);
    }
    return 0;
}
