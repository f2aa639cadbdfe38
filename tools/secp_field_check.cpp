// secp_field_check.cpp — drives secp256k1_host.hpp's field and point code
// for tests/test_secp_field.py (CPU, test infrastructure): one line of hex
// operands in, one line of normalized results out.
//   F a b      -> a*b  a^2  a+b  a-b  21a  a^-1 (a != 0)  (mod p; a, b < 2^256)
//   C a b      -> (a + a + a + a + a + a + a + a) * (b + b + b + b) - (a + a + a + a + a + a + a + a)
//                 (the largest magnitudes the point formulas feed fe_mul / fe_sub)
//   P k x y    -> k * (x, y) as 65-byte uncompressed hex, or "inf"
//   G k        -> k * G
//   T iters    -> best-of-20 microseconds of k * G, k * P and to65_pair (timing)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "../carbonado_amd/csrc/secp256k1_host.hpp"

using namespace chip::k1;

static void hex32(const std::string &h, uint8_t b[32]) {
    for (int i = 0; i < 32; ++i) b[i] = (uint8_t)std::stoi(h.substr(2 * i, 2), nullptr, 16);
}
static void put(const Fe &f) {
    uint8_t b[32];
    fe_to_be(f, b);
    for (int i = 0; i < 32; ++i) std::printf("%02x", b[i]);
    std::printf(" ");
}
static void put_pt(const Pt &p) {
    uint8_t o[65];
    if (!to65(p, o)) {
        std::printf("inf ");
        return;
    }
    for (int i = 0; i < 65; ++i) std::printf("%02x", o[i]);
    std::printf(" ");
}

int main() {
    std::string op;
    while (std::cin >> op) {
        if (op == "F" || op == "C") {
            std::string ha, hb;
            std::cin >> ha >> hb;
            uint8_t ab[32], bb[32];
            hex32(ha, ab), hex32(hb, bb);
            const Fe a = fe_from_be(ab), b = fe_from_be(bb);
            if (op == "F") {
                put(fe_mul(a, b)), put(fe_sqr(a)), put(fe_add(a, b)), put(fe_sub(a, b)), put(fe_mul21(a));
                if (!fe_is_zero(a)) put(fe_inv(a));
            } else {
                Fe a8 = a, b4 = b;
                for (int i = 0; i < 7; ++i) a8 = fe_add(a8, a);
                for (int i = 0; i < 3; ++i) b4 = fe_add(b4, b);
                put(fe_sub(fe_mul(a8, b4), a8)), put(fe_sqr(a8));
            }
        } else if (op == "P") {
            std::string hk, hx, hy;
            std::cin >> hk >> hx >> hy;
            uint8_t k[32], x[32], y[32];
            hex32(hk, k), hex32(hx, x), hex32(hy, y);
            put_pt(mul(k, fe_from_be(x), fe_from_be(y)));
        } else if (op == "T") {
            int iters;
            std::cin >> iters;
            uint8_t k[32], o[65], o2[65];
            for (int i = 0; i < 32; ++i) k[i] = (uint8_t)(i * 7 + 3);
            const Pt q = mul_g(k);
            auto best = [&](auto f) {
                double b = 1e30;
                for (int r = 0; r < 20; ++r) {
                    const auto t0 = std::chrono::steady_clock::now();
                    for (int i = 0; i < iters; ++i) f();
                    b = std::min(b, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
                }
                return b / iters * 1e6;
            };
            const double g = best([&] { Pt p = mul_g(k); k[3] ^= (uint8_t)p.x.v[0]; });
            const double m = best([&] { Pt p = mul(k, q.x, q.y); k[3] ^= (uint8_t)p.x.v[0]; });
            const double t = best([&] { to65_pair(q, q, o, o2); k[3] ^= o[9]; });
            std::printf("kG_us %.1f kP_us %.1f to65_pair_us %.1f ", g, m, t);
        } else if (op == "G") {
            std::string hk;
            std::cin >> hk;
            uint8_t k[32];
            hex32(hk, k);
            put_pt(mul_g(k));
        }
        std::printf("\n");
        std::fflush(stdout);
    }
    return 0;
}
