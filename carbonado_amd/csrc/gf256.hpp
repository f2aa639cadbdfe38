// gf256.hpp — host-side GF(2^8) arithmetic for the zfec plans.
//
// Field: GF(2^8) modulo x^8+x^4+x^3+x^2+1 (0x11D), generator 2 — the field of
// zfec's fec.c, which zfec-rs 0.1.0 (reference Cargo.toml:36) restates.
// Only the small k x k / m x k matrices live here; every byte of shard data is
// processed on the device (zfec_kernels.hip).
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace chip {

struct Gf256 {
    std::array<uint8_t, 512> exp{};
    std::array<int, 256> log{};
    Gf256() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = static_cast<uint8_t>(x);
            log[x] = i;
            x = (x << 1) ^ ((x & 0x80) ? 0x11D : 0);
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = -1;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t inv(uint8_t a) const { return a ? exp[255 - log[a]] : 0; }
    static const Gf256 &get() {
        static const Gf256 g;
        return g;
    }
};

// In-place inverse of an n x n matrix (row-major).  false if singular.
inline bool gf_invert(std::vector<uint8_t> &a, unsigned n) {
    const Gf256 &g = Gf256::get();
    std::vector<uint8_t> inv(n * n, 0);
    for (unsigned i = 0; i < n; ++i) inv[i * n + i] = 1;
    for (unsigned c = 0; c < n; ++c) {
        unsigned p = c;
        while (p < n && !a[p * n + c]) ++p;
        if (p == n) return false;
        if (p != c)
            for (unsigned j = 0; j < n; ++j) {
                std::swap(a[p * n + j], a[c * n + j]);
                std::swap(inv[p * n + j], inv[c * n + j]);
            }
        const uint8_t s = g.inv(a[c * n + c]);
        for (unsigned j = 0; j < n; ++j) {
            a[c * n + j] = g.mul(a[c * n + j], s);
            inv[c * n + j] = g.mul(inv[c * n + j], s);
        }
        for (unsigned r = 0; r < n; ++r) {
            const uint8_t f = a[r * n + c];
            if (r == c || !f) continue;
            for (unsigned j = 0; j < n; ++j) {
                a[r * n + j] ^= g.mul(f, a[c * n + j]);
                inv[r * n + j] ^= g.mul(f, inv[c * n + j]);
            }
        }
    }
    a.swap(inv);
    return true;
}

// m x k systematic encoding matrix of fec.c's fec_new(k, m): the Vandermonde
// matrix at the points {0, a^0, a^1, ..., a^(m-2)} right-multiplied by the
// inverse of its top k x k block (so rows 0..k-1 are the identity).
inline std::vector<uint8_t> zfec_enc_matrix(unsigned k, unsigned m) {
    const Gf256 &g = Gf256::get();
    std::vector<uint8_t> v(m * k, 0);
    v[0] = 1;  // point 0: 0^0 = 1, 0^c = 0
    for (unsigned r = 1; r < m; ++r)
        for (unsigned c = 0; c < k; ++c) v[r * k + c] = g.exp[((r - 1) * c) % 255];
    std::vector<uint8_t> top(v.begin(), v.begin() + k * k);
    gf_invert(top, k);  // a Vandermonde block at distinct points is never singular
    std::vector<uint8_t> e(m * k, 0);
    for (unsigned r = 0; r < m; ++r)
        for (unsigned c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (unsigned t = 0; t < k; ++t) acc ^= g.mul(v[r * k + t], top[t * k + c]);
            e[r * k + c] = acc;
        }
    return e;
}

}  // namespace chip
