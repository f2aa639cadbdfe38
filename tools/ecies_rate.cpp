// ecies_rate.cpp — per-object cost of the ECIES host stage on T threads
// (host_stages.cpp): ecies_prepare (two scalar multiplications + HKDF),
// ecies_encrypt of a 1-byte message, and the stream encrypt with a prepared
// key.  Thread-microseconds per operation (wall / ops per thread; every
// thread does N): flat in T when the threads do not contend.  Build (in tools/):
//   g++ -O2 -std=c++17 -I../carbonado_amd/csrc -I../include ecies_rate.cpp \
//       ../carbonado_amd/lib/obj/host_host_snap.cpp.o ../carbonado_amd/lib/obj/host_host_stages.cpp.o ../carbonado_amd/lib/obj/host_gcm_vaes.cpp.o -lcrypto -lpthread -o ecies_rate
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "host_stages.hpp"

using namespace chip::host;

int main(int argc, char **argv) {
    const int N = argc > 2 ? std::atoi(argv[2]) : 2000;
    uint8_t sk[32];
    for (int i = 0; i < 32; ++i) sk[i] = (uint8_t)(i + 1);
    uint8_t pub[65], peer[65];
    if (ecies_public_key(sk, pub) || ecies_peer(pub, 65, peer)) return 1;
    for (int T : {1, 4, 16}) {
        if (argc > 1 && T > std::atoi(argv[1])) break;
        auto run = [&](auto f) {
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(t); });
            for (auto &x : th) x.join();
            return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / N * 1e6;
        };
        const double a = run([&](int t) {
            EciesKey k;
            uint8_t e[32];
            std::memcpy(e, sk, 32);
            for (int i = 0; i < N; ++i) e[5] = (uint8_t)i, e[6] = (uint8_t)t, ecies_prepare(peer, e, &k);
        });
        const double b = run([&](int t) {
            uint8_t out[128], e[32], nonce[16] = {0}, in[1] = {7};
            uint64_t ol;
            std::memcpy(e, sk, 32);
            for (int i = 0; i < N; ++i)
                e[5] = (uint8_t)i, e[6] = (uint8_t)t, ecies_encrypt(pub, 65, e, nonce, in, 1, out, sizeof out, &ol);
        });
        const double c = run([&](int) {
            uint8_t out[128], nonce[16] = {0}, in[1] = {7};
            uint64_t ol;
            EciesKey k;
            ecies_prepare(peer, sk, &k);
            std::vector<uint8_t> win(SNAP_ECIES_WINDOW);
            for (int i = 0; i < N; ++i)
                ecies_encrypt_stream(nullptr, 0, nullptr, nonce, in, 1, false, out, sizeof out, &ol, win.data(),
                                     nullptr, nullptr, &k);
        });
        std::printf("threads %2d: thread-us per op: prepare %.1f  encrypt(1 B) %.1f  stream with prepared key %.1f\n",
                    T, a, b, c);
    }
    return 0;
}
