// key_probe.cpp — median us of the ECIES key steps on one thread
// (host_stages.cpp): ecies_peer of a 65-B key, ecies_derive_key (the decode's
// ECDH + HKDF), ecies_prepare (k*G and k*P).  Build (in tools/):
//   g++ -O2 -std=c++17 -I../carbonado_amd/csrc -I../include key_probe.cpp ../carbonado_amd/lib/obj/host_host_snap.cpp.o
//       ../carbonado_amd/lib/obj/host_host_stages.cpp.o ../carbonado_amd/lib/obj/host_host_stages_par.cpp.o
//       ../carbonado_amd/lib/obj/host_gcm_vaes.cpp.o -lcrypto -lpthread -o key_probe
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "host_stages.hpp"

using namespace chip::host;

template <class F>
static double med(int reps, F f) {
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const auto a = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
    return t[t.size() / 2];
}

int main() {
    uint8_t sk[32], eph[32], pub[65], epub[65], peer[65], key[32];
    for (int i = 0; i < 32; ++i) sk[i] = (uint8_t)(i + 1), eph[i] = (uint8_t)(i + 77);
    if (ecies_public_key(sk, pub) || ecies_public_key(eph, epub)) return 1;
    EciesKey k;
    std::printf("ecies_peer(65)   %7.2f us\n", med(2000, [&] { ecies_peer(pub, 65, peer); }));
    std::printf("ecies_derive_key %7.2f us\n", med(500, [&] { ecies_derive_key(sk, 32, epub, key); }));
    std::printf("ecies_prepare    %7.2f us\n", med(500, [&] { ecies_prepare(peer, eph, &k); }));
    return 0;
}
