// abi_latency.cpp — single-object encode()/decode() latency through the C-ABI
// alone (what the Rust crate's encode/decode cost once rerouted), without the
// Python mirror's buffer handling: the caller's buffers are allocated once
// and reused, as a service encoding segment after segment would.
//   g++ -std=c++17 -O2 tools/abi_latency.cpp -Iinclude -Lcarbonado_amd/lib -lcarbonado_hip \
//       -Wl,-rpath,'$ORIGIN/../carbonado_amd/lib' -o tools/abi_latency
//   abi_latency [REPS]        (levels 12 and 15, 1 KiB .. 16 MiB, median µs)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/carbonado_hip.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 50;
    uint8_t sk[32], pub[65];
    std::mt19937_64 rng(7);
    for (auto &x : sk) x = (uint8_t)rng();
    sk[0] &= 0x7f;
    if (chip_ecies_public_key(sk, pub) != CHIP_OK) return 1;
    std::printf("%5s %9s %10s %10s  (median of %d, C-ABI, buffers reused)\n", "level", "bytes", "enc_us", "dec_us",
                reps);
    for (int level : {12, 15, 4, 8}) {
        for (uint64_t n : {1024ull, 65536ull, 1ull << 20, 4ull << 20, 16ull << 20}) {
            std::vector<uint8_t> in(n), enc(chip_encode_max_len(n)), dec(n + (n >> 3) + 4096);
            for (auto &x : in) x = (uint8_t)rng();
            uint8_t hash[32];
            chip_encode_info info;
            uint64_t elen = 0, dlen = 0;
            auto encode = [&] {
                return chip_encode((uint8_t)level, pub, 65, nullptr, in.data(), n, enc.data(), enc.size(), &elen,
                                   hash, &info);
            };
            auto decode = [&] {
                return chip_decode(sk, 32, hash, 32, enc.data(), elen, info.padding_len, (uint8_t)level, dec.data(),
                                   dec.size(), &dlen);
            };
            if (encode() != CHIP_OK || decode() != CHIP_OK || dlen != n ||
                !std::equal(in.begin(), in.end(), dec.begin())) {
                std::printf("level %d n %llu: round trip failed\n", level, (unsigned long long)n);
                return 1;
            }
            std::vector<double> te, td;
            for (int r = 0; r < reps; ++r) {
                double t = now_us();
                encode();
                te.push_back(now_us() - t);
                t = now_us();
                decode();
                td.push_back(now_us() - t);
            }
            std::nth_element(te.begin(), te.begin() + reps / 2, te.end());
            std::nth_element(td.begin(), td.begin() + reps / 2, td.end());
            std::printf("%5d %9llu %10.1f %10.1f\n", level, (unsigned long long)n, te[reps / 2], td[reps / 2]);
        }
    }
    return 0;
}
