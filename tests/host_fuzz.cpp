// host_fuzz.cpp — test infrastructure (tests/test_host_asan.py builds it with
// AddressSanitizer + UndefinedBehaviorSanitizer and runs it).  Drives the
// library's HOST code — snappy framing, ECIES, the one-pass decrypt+unsnap,
// the 160-byte file header parser — with valid inputs and seeded mutations of
// them (bit flips, truncations, random chunk headers, random bytes), checking
// that every call either fails with a status or returns exactly the original
// bytes, and letting the sanitizers catch any out-of-bounds access.
//   host_fuzz SECONDS SEED
#include <openssl/evp.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../carbonado_amd/csrc/gcm_vaes.hpp"
#include "../carbonado_amd/csrc/host_stages.hpp"
#include "../include/carbonado_hip.h"

// file_container.cpp's file::encode/decode call the device pipeline, which is
// not linked here; the fuzzer never calls them.
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

using namespace chip::host;
using Bytes = std::vector<uint8_t>;

static std::mt19937_64 rng;
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

static Bytes compressible(size_t n) {
    Bytes out;
    while (out.size() < n) {
        const int kind = (int)rnd(4);
        if (kind == 0 || out.size() < 8) {
            for (uint64_t i = 0, k = 1 + rnd(200); i < k; ++i) out.push_back((uint8_t)rng());
        } else if (kind == 1) {
            out.insert(out.end(), 4 + rnd(3000), (uint8_t)rng());
        } else {
            const size_t dist = 1 + rnd(std::min<size_t>(out.size(), 70000));
            const size_t start = out.size() - dist;
            for (uint64_t i = 0, k = 4 + rnd(300); i < k; ++i) out.push_back(out[start + i]);
        }
    }
    out.resize(n);
    return out;
}

static Bytes mutate(const Bytes &in) {
    Bytes b = in;
    switch (rnd(4)) {
        case 0:  // bit flips
            for (uint64_t i = 0, k = 1 + rnd(4); i < k && !b.empty(); ++i) b[rnd(b.size())] ^= (uint8_t)(1u << rnd(8));
            break;
        case 1:  // truncation
            b.resize(rnd(b.size() + 1));
            break;
        case 2: {  // a random chunk header (type, 24-bit length) somewhere
            if (b.size() >= 4) {
                const size_t p = rnd(b.size() - 3);
                b[p] = (uint8_t)rng();
                b[p + 1] = (uint8_t)rng();
                b[p + 2] = (uint8_t)rng();
                b[p + 3] = (uint8_t)rnd(4);
            }
            break;
        }
        default:  // random bytes appended
            for (uint64_t i = 0, k = 1 + rnd(64); i < k; ++i) b.push_back((uint8_t)rng());
    }
    return b;
}

// memcmp with an empty range may see null pointers (std::vector::data() of an empty vector)
static bool same(const uint8_t *a, const uint8_t *b, size_t n) { return n == 0 || !std::memcmp(a, b, n); }

static int fails = 0;
#define EXPECT(c, ...)                             \
    do {                                           \
        if (!(c)) {                                \
            std::fprintf(stderr, "FAIL %s: ", #c); \
            std::fprintf(stderr, __VA_ARGS__);     \
            std::fprintf(stderr, "\n");            \
            ++fails;                               \
        }                                          \
    } while (0)

// gcm_vaes.cpp against OpenSSL's EVP AES-256-GCM (16-byte IV, no AAD): the
// message cut into random pieces (partial blocks, 256-B steps), in place or
// not, encrypt then decrypt; same ciphertext and tag
static void gcm_check(const Bytes &d) {
    using chip::host::Gcm;
    uint8_t key[32], iv[16], t1[16], t2[16];
    for (auto &x : key) x = (uint8_t)rng();
    for (auto &x : iv) x = (uint8_t)rng();
    const size_t n = d.size();
    Bytes ref(n + 16), got(d), back(n);
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int l = 0, f = 0;
    EXPECT(EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), nullptr, nullptr, nullptr) == 1 &&
               EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 16, nullptr) == 1 &&
               EVP_EncryptInit_ex(c, nullptr, nullptr, key, iv) == 1 &&
               EVP_EncryptUpdate(c, ref.data(), &l, d.data(), (int)n) == 1 &&
               EVP_EncryptFinal_ex(c, ref.data() + n, &f) == 1 &&
               EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, t1) == 1,
           "evp gcm n=%zu", n);
    EVP_CIPHER_CTX_free(c);
    auto pieces = [&](Gcm &g, const uint8_t *in, uint8_t *out) {
        for (size_t o = 0; o < n;) {
            const size_t k = std::min(n - o, (size_t)(rnd(3) == 0 ? rnd(17) : rnd(3) == 0 ? 256 * rnd(4) : rnd(2000)));
            EXPECT(g.update(in + o, k, out + o), "gcm update");
            o += k;
        }
    };
    Gcm g;
    g.init(key, iv, 16, true);
    pieces(g, got.data(), got.data());  // in place
    g.tag(t2);
    EXPECT(same(got.data(), ref.data(), n) && !std::memcmp(t1, t2, 16), "vaes gcm encrypt n=%zu", n);
    g.init(key, iv, 16, false);
    pieces(g, got.data(), back.data());
    g.tag(t2);
    EXPECT(same(back.data(), d.data(), n) && !std::memcmp(t1, t2, 16), "vaes gcm decrypt n=%zu", n);
    g.wipe();
}

// decompress with an exact-size buffer: an error, or exactly `orig`
static void snap_check(const Bytes &frame, const Bytes &orig, bool must_match) {
    uint64_t len = 0;
    const int sl = snap_decompressed_len(frame.data(), frame.size(), &len);
    Bytes out(sl == 0 ? len : orig.size());
    uint64_t got = 0;
    const int st = snap_decompress(frame.data(), frame.size(), out.data(), out.size(), &got);
    if (must_match) {
        EXPECT(st == 0 && got == orig.size() && same(out.data(), orig.data(), got), "valid frame, n=%zu",
               orig.size());
    } else if (st == 0) {
        // a mutation that still decodes passed every chunk's CRC: the original,
        // or a prefix of it (the frame cut at a chunk boundary: the framing
        // format has no end marker, so snap's FrameDecoder accepts it too)
        EXPECT(got <= orig.size() && same(out.data(), orig.data(), got), "mutated frame decoded to other bytes");
    }
    if (len > 0 && sl == 0) {  // a buffer one byte short: never written past
        Bytes small(len - 1);
        uint64_t g2 = 0;
        (void)snap_decompress(frame.data(), frame.size(), small.data(), small.size(), &g2);
    }
}

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? std::atof(argv[1]) : 10.0;
    rng.seed(argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 0xF022ull);
    const auto t0 = std::chrono::steady_clock::now();
    auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    uint8_t sk[32], pub[65];
    for (auto &x : sk) x = (uint8_t)rng();
    sk[0] &= 0x7f;
    EXPECT(ecies_public_key(sk, pub) == 0, "public key");
    if (chip::host::gcm_fast_available()) {  // GCM's length limit (2^36 - 32 bytes), as OpenSSL's
        chip::host::Gcm g;
        uint8_t k[32] = {1}, iv[16] = {2}, b[32] = {0};
        g.init(k, iv, 16, true);
        g.len = chip::host::GCM_MAX_BYTES - 32;
        EXPECT(g.update(b, 32, b), "gcm at its limit");
        EXPECT(!g.update(b, 1, b), "gcm past its limit");
    }
    long iters = 0;
    while (elapsed() < seconds) {
        ++iters;
        const size_t n = rnd(4) == 0 ? rnd(600000) : rnd(5000);
        const Bytes d = rnd(2) ? compressible(n) : [&] { Bytes r(n); for (auto &x : r) x = (uint8_t)rng(); return r; }();
        if (chip::host::gcm_fast_available()) gcm_check(d);
        // ring_copy (non-temporal stores into the staging ring): every length and both alignments
        {
            const size_t so = rnd(64), dof = rnd(64);
            Bytes src(n + so), dst(n + dof + 64, 0xA5);
            for (size_t i = 0; i < n; ++i) src[so + i] = d[i];
            ring_copy(dst.data() + dof, src.data() + so, n);
            EXPECT(std::memcmp(dst.data() + dof, d.data(), n) == 0, "ring_copy n=%zu", n);
            for (size_t i = 0; i < dof; ++i) EXPECT(dst[i] == 0xA5, "ring_copy wrote before dst");
            for (size_t i = dof + n; i < dst.size(); ++i) EXPECT(dst[i] == 0xA5, "ring_copy wrote past dst");
        }
        // snappy framing
        Bytes frame(snap_max_len(n));
        uint64_t fl = 0;
        EXPECT(snap_compress(d.data(), n, frame.data(), frame.size(), &fl) == 0, "compress n=%zu", n);
        frame.resize(fl);
        snap_check(frame, d, true);
        for (int k = 0; k < 4; ++k) snap_check(mutate(frame), d, false);
        // ECIES, and the one-pass decrypt + unsnap of a snappy frame
        const Bytes &pt = rnd(2) ? frame : d;
        Bytes ct(pt.size() + ECIES_OVERHEAD);
        uint64_t cl = 0;
        EXPECT(ecies_encrypt(pub, 65, nullptr, nullptr, pt.data(), pt.size(), ct.data(), ct.size(), &cl) == 0, "enc");
        ct.resize(cl);
        for (int k = 0; k < 3; ++k) {
            const Bytes bad = k == 0 ? ct : mutate(ct);
            Bytes out(pt.size() + 16);
            uint64_t ol = 0;
            const int st = ecies_decrypt(sk, 32, bad.data(), bad.size(), out.data(), out.size(), &ol);
            if (k == 0) EXPECT(st == 0 && ol == pt.size() && same(out.data(), pt.data(), ol), "dec");
            else if (st == 0) EXPECT(ol == pt.size() && same(out.data(), pt.data(), ol), "mutated ct decrypted");
            if (&pt == &frame) {
                Bytes o2(n + 16);
                uint64_t l2 = 0;
                const int s2 = ecies_decrypt_snap(sk, 32, bad.data(), bad.size(), o2.data(), o2.size(), &l2);
                if (k == 0) EXPECT(s2 == 0 && l2 == n && same(o2.data(), d.data(), n), "dec+unsnap");
                else if (s2 == 0) EXPECT(l2 == n && same(o2.data(), d.data(), n), "mutated dec+unsnap");
            }
        }
        // the pool's decrypt + unsnap against the one-pass one: a (maybe mutated) frame under a
        // valid tag, or a mutated envelope, with an exact, short or no output buffer
        if (frame.size() >= 200000) {
            const Bytes f2 = rnd(2) ? frame : mutate(frame);
            Bytes ct(f2.size() + ECIES_OVERHEAD);
            uint64_t cl = 0;
            EXPECT(ecies_encrypt(pub, 65, nullptr, nullptr, f2.data(), f2.size(), ct.data(), ct.size(), &cl) == 0,
                   "enc f2");
            ct.resize(cl);
            const Bytes env = rnd(4) ? ct : mutate(ct);
            const int mode = (int)rnd(3);  // 0 exact-ish, 1 short, 2 no buffer
            const uint64_t cap = mode == 0 ? n + 70000 : mode == 1 ? n / 2 : 0;
            Bytes o1(cap + 1), o2(cap + 1);
            uint64_t l1 = 0, l2 = 0;
            const int s1 = ecies_decrypt_snap(sk, 32, env.data(), env.size(), mode == 2 ? nullptr : o1.data(), cap, &l1);
            const int s2 = ecies_decrypt_snap_par(sk, 32, env.data(), env.size(), mode == 2 ? nullptr : o2.data(), cap,
                                                  &l2);
            EXPECT(s1 == s2, "par dec status %d vs %d n=%zu mode=%d", s2, s1, n, mode);
            if (s1 == s2 && (s1 == 0 || s1 == CHIP_ERR_BUFFER_TOO_SMALL)) EXPECT(l1 == l2, "par dec len");
            if (s1 == 0 && s2 == 0) EXPECT(same(o1.data(), o2.data(), l1), "par dec bytes");
        }
        // one-pass ECIES (|snappy) with and without a chunk sink: the same bytes as
        // snap_compress + ecies_encrypt; chunks [1, filled) at their slots, nothing else written
        {
            uint8_t eph[32], iv[16];
            for (auto &x : eph) x = (uint8_t)rng();
            eph[0] &= 0x7f;
            eph[31] |= 1;
            for (auto &x : iv) x = (uint8_t)rng();
            const bool snap = rnd(2);
            const Bytes &plain = snap ? frame : d;
            Bytes ref(plain.size() + ECIES_OVERHEAD);
            uint64_t rl = 0;
            EXPECT(ecies_encrypt(pub, 65, eph, iv, plain.data(), plain.size(), ref.data(), ref.size(), &rl) == 0,
                   "ref enc");
            const uint64_t cap = (snap ? snap_max_len(n) : n) + ECIES_OVERHEAD;
            Bytes win(SNAP_ECIES_WINDOW), out(cap);
            // complete: the sink takes every chunk the output touches (and may be the only output)
            const bool complete = rnd(2);
            const uint64_t nd = complete ? (cap + 1023) / 1024 + rnd(3) : rl / 1024 + rnd(3);
            std::vector<uint64_t> coff(nd);
            for (uint64_t i = 0; i < nd; ++i) coff[i] = 8 + 1088 * i + 64 * rnd(2) * (i > 0);
            Bytes strm(8 + 1088 * (nd + 1), 0xA5);
            const uint64_t zl = 1024 * rng() % (1ull << 40);
            const ChunkSink sink{strm.data(), coff.data(), nd, complete, zl};
            uint64_t ol = 0, filled = 0;
            const bool with_sink = rnd(2) && nd;
            const bool no_out = with_sink && complete && rnd(2);
            EXPECT(ecies_encrypt_stream(pub, 65, eph, iv, d.data(), n, snap, no_out ? nullptr : out.data(), cap, &ol,
                                        win.data(), with_sink ? &sink : nullptr, &filled) == 0, "stream enc");
            EXPECT(ol == rl && (no_out || same(out.data(), ref.data(), rl)), "stream enc bytes n=%zu snap=%d", n,
                   (int)snap);
            if (with_sink) {
                Bytes want(strm.size(), 0xA5);
                Bytes padded(ref.begin(), ref.begin() + rl);
                padded.resize((rl + 1023) / 1024 * 1024, 0);
                if (complete) {
                    for (int b = 0; b < 8; ++b) want[b] = (uint8_t)(zl >> (8 * b));
                    EXPECT(filled == (rl + 1023) / 1024, "complete filled %llu", (unsigned long long)filled);
                }
                for (uint64_t i = complete ? 0 : 1; i < filled; ++i)
                    std::memcpy(want.data() + coff[i], padded.data() + 1024 * i, 1024);
                EXPECT(filled <= std::max<uint64_t>(1, nd) && 1024 * filled <= rl + 1023, "filled %llu",
                       (unsigned long long)filled);
                EXPECT(strm == want, "sink chunks n=%zu snap=%d complete=%d filled=%llu", n, (int)snap,
                       (int)complete, (unsigned long long)filled);
                if (complete) {  // gather_chunks reads the output back from the slots
                    Bytes back(rl);
                    gather_chunks(back.data(), strm.data(), coff.data(), rl);
                    EXPECT(back == Bytes(ref.begin(), ref.begin() + rl), "gather_chunks");
                }
            }
            {  // one object's stage on the worker pool (from STAGE_PAR_MIN; below it, the one-thread paths)
                Bytes pout(cap);
                uint64_t pl = 0;
                const int ps = snap ? ecies_encrypt_par(pub, 65, eph, iv, d.data(), n, pout.data(), cap, &pl, win.data())
                                    : ecies_encrypt_par_plain(pub, 65, eph, iv, d.data(), n, pout.data(), cap, &pl);
                EXPECT(ps == 0, "par enc");
                EXPECT(pl == rl && same(pout.data(), ref.data(), rl), "par enc bytes n=%zu snap=%d", n, (int)snap);
                if (!snap) {  // and back, maybe through a flipped byte
                    Bytes env(pout.begin(), pout.begin() + pl);
                    if (rnd(2)) env[rnd(env.size())] ^= (uint8_t)(1u << rnd(8));
                    Bytes o1(n + 1), o2(n + 1);
                    uint64_t l1 = 0, l2 = 0;
                    const int s1 = ecies_decrypt(sk, 32, env.data(), env.size(), o1.data(), o1.size(), &l1);
                    const int s2 = ecies_decrypt_par(sk, 32, env.data(), env.size(), o2.data(), o2.size(), &l2);
                    EXPECT(s1 == s2 && (s1 != 0 || (l1 == l2 && same(o1.data(), o2.data(), l1))),
                           "par dec plain %d vs %d n=%zu", s2, s1, n);
                }
            }
        }
        // snap_compress_stream: the frame of snap_compress, chunks [0, filled) at their slots
        {
            const bool complete = rnd(2);
            const uint64_t m = snap_max_len(n);
            const uint64_t nd = complete ? (m + 1023) / 1024 + rnd(3) : fl / 1024 + rnd(3);
            std::vector<uint64_t> coff(nd);
            for (uint64_t i = 0; i < nd; ++i) coff[i] = 8 + 1088 * i + 64 * rnd(2) * (i > 0);
            Bytes strm(8 + 1088 * (nd + 1), 0xA5), win(SNAP_ECIES_WINDOW), out2(m + 1);
            const uint64_t zl = 1024 * (1 + rnd(1000));
            const ChunkSink sink{strm.data(), coff.data(), nd, complete, zl};
            const bool with_sink = rnd(2) && nd;
            const bool no_out = with_sink && complete && rnd(2);
            uint64_t ol = 0, filled = 0;
            EXPECT(snap_compress_stream(d.data(), n, no_out ? nullptr : out2.data(), out2.size(), &ol, win.data(),
                                        with_sink ? &sink : nullptr, &filled) == 0, "snap stream n=%zu", n);
            EXPECT(ol == fl && (no_out || same(out2.data(), frame.data(), fl)), "snap stream bytes n=%zu", n);
            if (with_sink && n) {
                Bytes want(strm.size(), 0xA5);
                Bytes padded(frame.begin(), frame.end());
                padded.resize((fl + 1023) / 1024 * 1024, 0);
                if (complete) {
                    for (int b = 0; b < 8; ++b) want[b] = (uint8_t)(zl >> (8 * b));
                    EXPECT(filled == (fl + 1023) / 1024, "snap complete filled");
                }
                for (uint64_t i = 0; i < filled; ++i) std::memcpy(want.data() + coff[i], padded.data() + 1024 * i, 1024);
                EXPECT(strm == want, "snap sink chunks n=%zu complete=%d filled=%llu", n, (int)complete,
                       (unsigned long long)filled);
            }
        }
        // the 160-byte file header
        chip_header h{};
        uint8_t hash[32], meta[8], aux[32], bytes[CHIP_HEADER_LEN];
        for (auto &x : hash) x = (uint8_t)rng();
        for (auto &x : meta) x = (uint8_t)rng();
        for (auto &x : aux) x = (uint8_t)rng();
        EXPECT(chip_header_new(sk, 32, pub, 65, hash, 32, (uint8_t)rnd(16), (uint8_t)rng(), (uint32_t)rng(),
                               (uint32_t)rng(), rnd(2) ? meta : nullptr, aux, &h) == 0, "header new");
        EXPECT(chip_header_to_bytes(&h, bytes) == 0, "header bytes");
        chip_header back{};
        EXPECT(chip_header_parse(bytes, CHIP_HEADER_LEN, &back) == 0 && !std::memcmp(&back.hash, &h.hash, 32),
               "header parse");
        const Bytes good(bytes, bytes + CHIP_HEADER_LEN);
        for (int k = 0; k < 4; ++k) {
            const Bytes bad = mutate(good);
            chip_header x{};
            (void)chip_header_parse(bad.data(), bad.size(), &x);
        }
    }
    std::printf("host_fuzz: %ld iterations in %.1f s, %d failures\n", iters, elapsed(), fails);
    return fails ? 1 : 0;
}
