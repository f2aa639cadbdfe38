// host_encode_probe.cpp — where a host thread's time goes in encode()'s
// host stages at level 15 (diagnostic): per 16 MiB random
// object, CRC-32C alone, snap_compress, ecies_encrypt, the one-pass
// ecies_encrypt_stream without and with a chunk sink, and a plain memcpy;
// one thread, then T threads each on its own objects.
//   g++ -std=c++17 -O3 tools/host_encode_probe.cpp carbonado_amd/csrc/host_snap.cpp carbonado_amd/csrc/host_stages.cpp carbonado_amd/csrc/gcm_vaes.cpp \
//       carbonado_amd/csrc/file_container.cpp -Iinclude -lcrypto -lpthread -o tools/host_encode_probe
//   host_encode_probe [THREADS] [REPS]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <thread>
#include <vector>

#include "../carbonado_amd/csrc/host_stages.hpp"
#include "../include/carbonado_hip.h"

extern "C" {  // file_container.cpp's device entry points are never called here
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

using namespace chip::host;

struct Obj {  // one thread's buffers
    std::vector<uint8_t> in, frame, ct, win, strm;
    std::vector<uint64_t> coff;
    explicit Obj(uint64_t n, uint64_t seed) : in(n), frame(snap_max_len(n)), ct(snap_max_len(n) + ECIES_OVERHEAD),
                                              win(SNAP_ECIES_WINDOW) {
        std::mt19937_64 r(seed);
        for (size_t i = 0; i < n; i += 8) {
            const uint64_t v = r();
            std::memcpy(in.data() + i, &v, std::min<size_t>(8, n - i));
        }
        const uint64_t nd = (ct.size() + 1023) / 1024;
        coff.resize(nd);
        for (uint64_t i = 0; i < nd; ++i) coff[i] = 8 + 1088 * i;
        strm.assign(8 + 1088 * (nd + 1), 0);
    }
};

int main(int argc, char **argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 16;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 4;
    const uint64_t n = 16u << 20;
    uint8_t sk[32], pub[65], eph[32], iv[16];
    for (int i = 0; i < 32; ++i) sk[i] = eph[i] = (uint8_t)(i + 1);
    for (int i = 0; i < 16; ++i) iv[i] = (uint8_t)i;
    if (ecies_public_key(sk, pub)) return 1;
    using Fn = std::function<void(Obj &)>;
    const std::pair<const char *, Fn> cases[] = {
        {"crc32c", [&](Obj &o) { (void)crc32c(o.in.data(), n); }},
        {"memcpy 16 MiB", [&](Obj &o) { std::memcpy(o.frame.data(), o.in.data(), n); }},
        {"snap_compress", [&](Obj &o) { uint64_t l; (void)snap_compress(o.in.data(), n, o.frame.data(), o.frame.size(), &l); }},
        {"ecies_encrypt (of the input)", [&](Obj &o) { uint64_t l; (void)ecies_encrypt(pub, 65, eph, iv, o.in.data(), n, o.ct.data(), o.ct.size(), &l); }},
        {"snap + ecies two-pass", [&](Obj &o) {
             uint64_t l, c;
             (void)snap_compress(o.in.data(), n, o.frame.data(), o.frame.size(), &l);
             (void)ecies_encrypt(pub, 65, eph, iv, o.frame.data(), l, o.ct.data(), o.ct.size(), &c);
         }},
        {"one pass, no sink", [&](Obj &o) { uint64_t l, f; (void)ecies_encrypt_stream(pub, 65, eph, iv, o.in.data(), n, true, o.ct.data(), o.ct.size(), &l, o.win.data(), nullptr, &f); }},
        {"one pass + chunk sink", [&](Obj &o) {
             const ChunkSink s{o.strm.data(), o.coff.data(), o.coff.size()};
             uint64_t l, f;
             (void)ecies_encrypt_stream(pub, 65, eph, iv, o.in.data(), n, true, o.ct.data(), o.ct.size(), &l, o.win.data(), &s, &f);
         }},
    };
    for (int threads : {1, T}) {
        std::vector<Obj> objs;
        for (int t = 0; t < threads; ++t) objs.emplace_back(n, 77 + t);
        for (const auto &c : cases) {
            auto run = [&](int t) { for (int r = 0; r < reps; ++r) c.second(objs[t]); };
            run(0);  // touch
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> pool;
            for (int t = 0; t < threads; ++t) pool.emplace_back(run, t);
            for (auto &th : pool) th.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::printf("%-30s threads %3d: %7.2f GiB/s aggregate, %6.2f per thread\n", c.first, threads,
                        threads * reps * (double)n / s / (1 << 30), reps * (double)n / s / (1 << 30));
            std::fflush(stdout);
        }
    }
    return 0;
}
