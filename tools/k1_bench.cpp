// k1_bench.cpp — host timing of the secp256k1 scalar multiplications the
// ECIES host stage runs per object (carbonado_amd/csrc/secp256k1_host.hpp):
// k*G (ephemeral public key), k*P (shared point), the affine conversion.
// Calibration tool (not product code).   g++ -O3 -std=c++17 k1_bench.cpp
#include <chrono>
#include <cstdio>
#include <random>

#include "../carbonado_amd/csrc/secp256k1_host.hpp"

using namespace chip::k1;

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937_64 rng(7);
    uint8_t k[32], out[65];
    for (auto &b : k) b = (uint8_t)rng();
    k[0] &= 0x7f;
    (void)gtable();
    Fe x = gx(), y = gy();
    auto t0 = std::chrono::steady_clock::now();
    uint64_t sink = 0;
    for (int i = 0; i < n; ++i) {
        k[31] = (uint8_t)i;
        Pt r = mul_g(k);
        sink += r.x.v[0];
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        k[31] = (uint8_t)i;
        Pt r = mul(k, x, y);
        sink += r.x.v[0];
    }
    auto t2 = std::chrono::steady_clock::now();
    Pt p = mul_g(k);
    for (int i = 0; i < n; ++i) {
        p.z.v[0] ^= (uint64_t)i;
        sink += to65(p, out) ? out[5] : 0;
    }
    auto t3 = std::chrono::steady_clock::now();
    Fe a = gx();
    for (int i = 0; i < n * 100; ++i) a = fe_mul(a, y);
    auto t4 = std::chrono::steady_clock::now();
    auto us = [&](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count() / n; };
    printf("k*G %.1f us  k*P %.1f us  to65 %.1f us  fe_mul %.1f ns  (%llu)\n", us(t0, t1), us(t1, t2), us(t2, t3),
           us(t3, t4) * 1e3 / 100, (unsigned long long)(sink + a.v[0]));
    return 0;
}
