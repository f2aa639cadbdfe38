// host_stages_par.cpp — one object's ECIES stage on a few threads
// (encode()/decode() of a single object at Ecies, encoding.rs:30-36 and
// decoding.rs:62-77): a persistent StagePool, AES-GCM split into 16-B aligned
// pieces whose GHASH parts are joined (gcm_vaes.hpp), the snappy blocks
// compressed or decoded on every thread.  Same bytes and statuses as the
// one-thread paths of host_stages.cpp, which every function here falls back
// to (small object, no VAES, busy pool, a message past GCM's length limit).
#include "host_stages.hpp"
#include "gcm_vaes.hpp"
#include "snap_internal.hpp"

#include <openssl/crypto.h>
#include <openssl/rand.h>

#include <immintrin.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/carbonado_hip.h"

namespace chip {
namespace host {

// ------------------------------------------- one object's stage on a few threads
namespace {

// Persistent workers for one object's host stage (chip_encode).  start(f)
// runs f(1) .. f(W) on the workers; wait() returns once they are done.  A
// caller that finds the pool busy (another thread's object) or in a forked
// child takes the one-thread path instead.
class StagePool {
  public:
    static StagePool &get() {
        static StagePool *p = new StagePool();  // never destroyed: workers park on the condvar at exit
        return *p;
    }
    int workers() const { return workers_; }
    bool try_acquire() { return workers_ > 0 && getpid() == pid_ && job_.try_lock(); }
    // Workers spin for a short while after each job before they park, so the
    // next job of the same call (an object takes two or three) starts without
    // a futex wake-up.
    void start(std::function<void(int)> f) {
        f_ = std::move(f);
        pending_.store(workers_, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    void wait() {
        for (int i = 0; pending_.load(std::memory_order_acquire) != 0; ++i) {
            if (i < SPIN) {
                _mm_pause();
            } else {
                std::unique_lock<std::mutex> lk(mu_);
                done_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
            }
        }
        f_ = nullptr;
    }
    void release() { job_.unlock(); }

  private:
    static constexpr int SPIN = 1 << 15;  // ~0.1 ms of pause instructions
    StagePool() {
        // the calling thread + up to 15 workers, no more than the machine's
        // hardware threads (r11zzd: 16 against 8, level 15 of 4 MiB of text
        // 608-647 -> 407-438 us); CHIP_STAGE_THREADS=1: one thread
        const int hw = (int)std::thread::hardware_concurrency();
        int t = std::max(1, std::min(16, hw > 0 ? hw : 8));
        if (const char *e = std::getenv("CHIP_STAGE_THREADS")) t = std::max(1, std::min(32, std::atoi(e)));
        workers_ = t - 1;
        pid_ = getpid();
        for (int i = 1; i <= workers_; ++i) std::thread([this, i] { run(i); }).detach();
    }
    void run(int i) {
        uint64_t seen = 0;
        for (;;) {
            for (int k = 0; gen_.load(std::memory_order_acquire) == seen; ++k) {
                if (k < SPIN) {
                    _mm_pause();
                } else {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                }
            }
            seen = gen_.load(std::memory_order_acquire);
            f_(i);  // f_ stays put until every worker has counted itself done
            if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_.notify_one();
            }
        }
    }
    int workers_ = 0;
    pid_t pid_ = 0;
    std::mutex job_, mu_;
    std::condition_variable cv_, done_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::function<void(int)> f_;
};

// A calling thread's scratch of the pooled stage (compressed blocks, or a
// plaintext buffer): kept for the next object up to SCRATCH_KEEP bytes, freed
// on return beyond that, so one huge object does not pin its size per thread.
constexpr size_t SCRATCH_KEEP = 64u << 20;
struct ScratchCap {
    std::vector<uint8_t> &v;
    ~ScratchCap() {
        if (v.size() > SCRATCH_KEEP) std::vector<uint8_t>().swap(v);
    }
};

// AES-GCM of m contiguous bytes in T 16-B aligned pieces, one per pool thread
// (the caller holds the pool); the pieces' GHASH joined into msg.  Each part's
// Gcm starts its own byte count at 0, so the message's limit (GCM_MAX_BYTES:
// past it the 32-bit block counter wraps and keystream repeats) is the
// caller's to check on the whole m first; false if a part's update refused.
bool gcm_parts(StagePool &pool, Gcm &msg, const uint8_t *in, uint8_t *out, uint64_t m) {
    const int T = std::min(pool.workers() + 1, 32);
    const uint64_t S = ((m + T - 1) / T + 15) / 16 * 16;
    uint8_t ys[32][16];
    std::atomic<bool> ok{true};
    auto part = [&](int w) {
        const uint64_t a = (uint64_t)w * S;
        if (a >= m) return;
        const uint64_t b = std::min(m, a + S);
        Gcm g;
        g.init_part(msg, a);
        if (!g.update(in + a, b - a, out + a)) ok.store(false, std::memory_order_relaxed);
        g.part_ghash(ys[w]);
        g.wipe();
    };
    pool.start(part);
    part(0);
    pool.wait();
    const uint64_t blocks = (m + 15) / 16;
    for (int w = 0; w < T && (uint64_t)w * S < m; ++w)
        msg.join_part(ys[w], blocks - (std::min(m, (uint64_t)(w + 1) * S) + 15) / 16);
    OPENSSL_cleanse(ys, sizeof ys);
    return ok.load();
}

// n bytes at p wiped on every pool thread
void wipe_parts(StagePool &pool, uint8_t *p, uint64_t n) {
    const int T = std::min(pool.workers() + 1, 32);
    const uint64_t S = (n + T - 1) / T;
    auto w = [&](int i) {
        const uint64_t a = (uint64_t)i * S;
        if (a < n) OPENSSL_cleanse(p + a, std::min(S, n - a));
    };
    pool.start(w);
    w(0);
    pool.wait();
}

}  // namespace

int ecies_encrypt_par(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk, const uint8_t *nonce,
                      const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                      uint8_t *window) {
    StagePool &pool = StagePool::get();
    if (n < STAGE_PAR_MIN || !out || cap < snap_max_len(n) + ECIES_OVERHEAD || !gcm_vaes_on() ||
        snap_max_len(n) > GCM_MAX_BYTES || !pool.try_acquire())
        return ecies_encrypt_stream(pubkey, pubkey_len, eph_sk, nonce, in, n, true, out, cap, out_len, window, nullptr,
                                    nullptr);
    struct Block {
        uint8_t hdr[8];
        const uint8_t *body;
        size_t blen;
    };
    const int T = std::min(pool.workers() + 1, 32);
    const uint64_t nb = (n + MAX_BLOCK - 1) / MAX_BLOCK;
    static thread_local std::vector<uint8_t> t_scr;  // one compressed block per slot
    if (t_scr.size() < nb * MAX_COMPRESS_BLOCK) t_scr.resize(nb * MAX_COMPRESS_BLOCK);
    ScratchCap cap_scr{t_scr};
    uint8_t *scr = t_scr.data();
    std::vector<Block> blk(nb);
    std::vector<uint64_t> boff(nb);  // frame offset of each block's chunk header
    std::atomic<uint64_t> next{0};
    EciesKey key;
    // 1: the snappy blocks on every thread, the key agreement's two scalar
    // multiplications first: k·G here, k·P on one worker
    auto compress = [&] {
        for (uint64_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nb;) {
            const uint64_t o = j * MAX_BLOCK;
            const size_t len = (size_t)std::min<uint64_t>(MAX_BLOCK, n - o);
            blk[j].blen = snap_block(in + o, len, blk[j].hdr, scr + j * MAX_COMPRESS_BLOCK, &blk[j].body);
        }
    };
    bool compressed = false;
    auto run2 = [&](const std::function<void(int)> &f) {
        pool.start([&](int w) {
            if (w == 1) f(1);
            compress();
        });
        f(0);
        compress();
        pool.wait();  // blk is this thread's from here (the pool's mutex orders it)
        compressed = true;
    };
    uint8_t peer[65];
    int key_st = ecies_peer(pubkey, pubkey_len, peer);
    if (key_st == CHIP_OK) key_st = ecies_prepare_with(peer, eph_sk, &key, run2);
    if (key_st == CHIP_OK && !compressed) key_st = CHIP_ERR_ECIES;  // (run2 is called on every success)
    uint8_t *iv = out + 65;
    if (key_st == CHIP_OK) {
        std::memcpy(out, key.eph_pub, 65);
        if (nonce) std::memcpy(iv, nonce, 16);
        else if (RAND_bytes(iv, 16) != 1) key_st = CHIP_ERR_ECIES;
    }
    if (key_st != CHIP_OK) {
        pool.release();
        ecies_key_wipe(&key);
        return key_st;
    }
    uint64_t mf = sizeof(STREAM_ID);
    for (uint64_t j = 0; j < nb; ++j) {
        boff[j] = mf;
        mf += 8 + blk[j].blen;
    }
    Gcm msg;
    msg.init(key.key, iv, 16, true);
    ecies_key_wipe(&key);
    // 2: AES-GCM over T 16-B aligned pieces of the frame, one per thread, each
    // reading its bytes from the identifier, chunk headers and bodies in place
    uint8_t *ct = out + 97;
    const uint64_t S = ((mf + T - 1) / T + 15) / 16 * 16;
    uint8_t ys[32][16];
    std::atomic<bool> part_ok{true};
    auto part = [&](int w) {
        const uint64_t a = (uint64_t)w * S;
        if (a >= mf) return;
        const uint64_t b = std::min(mf, a + S);
        Gcm g;
        g.init_part(msg, a);
        uint64_t pos = a;
        uint64_t j = std::upper_bound(boff.begin(), boff.end(), pos) - boff.begin();  // blocks starting <= pos
        j = j ? j - 1 : 0;
        while (pos < b) {
            const uint8_t *src;
            uint64_t end;
            if (pos < sizeof(STREAM_ID)) {
                src = STREAM_ID + pos;
                end = sizeof(STREAM_ID);
            } else {
                while (j + 1 < nb && boff[j + 1] <= pos) ++j;
                if (pos < boff[j] + 8) {
                    src = blk[j].hdr + (pos - boff[j]);
                    end = boff[j] + 8;
                } else {
                    src = blk[j].body + (pos - boff[j] - 8);
                    end = boff[j] + 8 + blk[j].blen;
                }
            }
            const uint64_t len = std::min(end, b) - pos;
            if (!g.update(src, len, ct + pos)) part_ok.store(false, std::memory_order_relaxed);
            pos += len;
        }
        g.part_ghash(ys[w]);
        g.wipe();
    };
    pool.start(part);
    part(0);
    pool.wait();
    pool.release();
    const uint64_t blocks = (mf + 15) / 16;
    for (int w = 0; w < T && (uint64_t)w * S < mf; ++w)
        msg.join_part(ys[w], blocks - (std::min(mf, (uint64_t)(w + 1) * S) + 15) / 16);
    msg.tag_joined(mf, out + 81);
    msg.wipe();
    OPENSSL_cleanse(ys, sizeof ys);
    if (!part_ok.load()) return CHIP_ERR_ECIES;
    *out_len = mf + ECIES_OVERHEAD;
    return CHIP_OK;
}

static int snap_frames_par(StagePool &pool, const uint8_t *P, uint64_t m, uint8_t *out, uint64_t cap,
                           uint64_t *out_len);

int snap_compress_par(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    StagePool &pool = StagePool::get();
    if (n < STAGE_PAR_MIN || !out || cap < snap_max_len(n) || !pool.try_acquire())
        return snap_compress(in, n, out, cap, out_len);
    struct Hold {
        StagePool &p;
        ~Hold() { p.release(); }
    } hold{pool};
    struct Block {
        uint8_t hdr[8];
        const uint8_t *body;
        size_t blen;
    };
    const uint64_t nb = (n + MAX_BLOCK - 1) / MAX_BLOCK;
    static thread_local std::vector<uint8_t> t_scr;  // one compressed block per slot
    if (t_scr.size() < nb * MAX_COMPRESS_BLOCK) t_scr.resize(nb * MAX_COMPRESS_BLOCK);
    ScratchCap cap_scr{t_scr};
    uint8_t *scr = t_scr.data();
    std::vector<Block> blk(nb);
    std::atomic<uint64_t> next{0};
    // 1: the blocks on every thread (FrameEncoder's rule per block: snap_block)
    auto compress = [&](int) {
        for (uint64_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nb;) {
            const uint64_t o = j * MAX_BLOCK;
            const size_t len = (size_t)std::min<uint64_t>(MAX_BLOCK, n - o);
            blk[j].blen = snap_block(in + o, len, blk[j].hdr, scr + j * MAX_COMPRESS_BLOCK, &blk[j].body);
        }
    };
    pool.start(compress);
    compress(0);
    pool.wait();
    // 2: the frame: identifier, then each block's header and body at its offset, on every thread
    std::vector<uint64_t> boff(nb);
    uint64_t mf = sizeof(STREAM_ID);
    for (uint64_t j = 0; j < nb; ++j) {
        boff[j] = mf;
        mf += 8 + blk[j].blen;
    }
    std::memcpy(out, STREAM_ID, sizeof(STREAM_ID));
    next.store(0, std::memory_order_relaxed);
    auto place = [&](int) {
        for (uint64_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nb;) {
            std::memcpy(out + boff[j], blk[j].hdr, 8);
            std::memcpy(out + boff[j] + 8, blk[j].body, blk[j].blen);
        }
    };
    pool.start(place);
    place(0);
    pool.wait();
    *out_len = mf;
    return CHIP_OK;
}

int snap_decompress_par(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    StagePool &pool = StagePool::get();
    if (n < STAGE_PAR_MIN || !pool.try_acquire()) return snap_decompress(in, n, out, cap, out_len);
    struct Hold {
        StagePool &p;
        ~Hold() { p.release(); }
    } hold{pool};
    return snap_frames_par(pool, in, n, out, cap, out_len);
}

void par_for(int parts, const std::function<void(int)> &f) {
    StagePool &pool = StagePool::get();
    if (parts <= 1 || !pool.try_acquire()) {
        for (int i = 0; i < parts; ++i) f(i);
        return;
    }
    std::atomic<int> next{0};
    auto run = [&](int) {
        for (int i; (i = next.fetch_add(1, std::memory_order_relaxed)) < parts;) f(i);
    };
    pool.start(run);
    run(0);
    pool.wait();
    pool.release();
}

bool ecies_par_eligible(uint64_t n) {
    return n >= ECIES_OVERHEAD + STAGE_PAR_MIN && n - ECIES_OVERHEAD <= GCM_MAX_BYTES && gcm_vaes_on();
}

// A snappy frame stream P[0, m) decoded on the pool (held by the caller):
// snap_walk's size pass over the chunk headers, then the chunks (CRC, raw
// copy or block decode) on every thread.  Status order as snap_decompress:
// framing errors, then a short `out` (the required size in *out_len), then
// CRC / block errors.
static int snap_frames_par(StagePool &pool, const uint8_t *P, uint64_t m, uint8_t *out, uint64_t cap,
                           uint64_t *out_len) {
    struct Chunk {
        uint64_t src, dl, doff, ulen;
        uint32_t want;
        uint8_t ty;
    };
    std::vector<Chunk> ch;
    ch.reserve(m / MAX_BLOCK + 2);
    uint64_t s = 0, d = 0;
    bool ident = false;
    int frame = CHIP_OK;
    while (s < m) {
        if (m - s < 4) { frame = CHIP_ERR_SNAP; break; }
        const uint8_t ty = P[s];
        const uint64_t clen = (uint64_t)P[s + 1] | ((uint64_t)P[s + 2] << 8) | ((uint64_t)P[s + 3] << 16);
        s += 4;
        if (clen > m - s) { frame = CHIP_ERR_SNAP; break; }
        const uint8_t *body = P + s;
        if (!ident && ty != 0xFF) { frame = CHIP_ERR_SNAP; break; }
        if (ty == 0xFF) {
            if (clen != 6 || std::memcmp(body, STREAM_ID + 4, 6) != 0) { frame = CHIP_ERR_SNAP; break; }
            ident = true;
        } else if (ty == 0x00 || ty == 0x01) {
            if (clen < 4) { frame = CHIP_ERR_SNAP; break; }
            Chunk c{s + 4, clen - 4, d, clen - 4, 0, ty};
            std::memcpy(&c.want, body, 4);
            if (ty == 0x01) {
                if (c.dl > MAX_BLOCK) { frame = CHIP_ERR_SNAP; break; }
            } else {
                size_t used;
                if (!get_varint(body + 4, c.dl, &c.ulen, &used) || c.ulen > MAX_BLOCK) { frame = CHIP_ERR_SNAP; break; }
            }
            ch.push_back(c);
            d += c.ulen;
        } else if (ty >= 0x02 && ty <= 0x7F) {
            frame = CHIP_ERR_SNAP;  // reserved unskippable
            break;
        }  // 0x80..0xFE: padding / reserved skippable
        s += clen;
    }
    if (frame != CHIP_OK || d > cap || (d && !out)) {
        if (frame != CHIP_OK) return frame;
        *out_len = d;
        return CHIP_ERR_BUFFER_TOO_SMALL;
    }
    // 3: the chunks (CRC, raw copy or block decode) on every thread
    std::atomic<uint64_t> next{0};
    std::atomic<bool> bad{false};
    auto content = [&](int) {
        for (uint64_t j; (j = next.fetch_add(1, std::memory_order_relaxed)) < ch.size();) {
            const Chunk &c = ch[j];
            const uint8_t *data = P + c.src;
            bool ok;
            if (c.ty == 0x01) {
                ok = crc_masked(data, c.dl) == c.want;
                if (ok) std::memcpy(out + c.doff, data, c.dl);
            } else {
                size_t got;
                ok = decompress_raw(data, c.dl, out + c.doff, c.ulen, &got) && got == c.ulen &&
                     crc_masked(out + c.doff, c.ulen) == c.want;
            }
            if (!ok) bad.store(true, std::memory_order_relaxed);
        }
    };
    pool.start(content);
    content(0);
    pool.wait();
    if (bad.load()) return CHIP_ERR_SNAP;
    *out_len = d;
    return CHIP_OK;
}


int ecies_decrypt_snap_par(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n,
                           uint8_t *out, uint64_t cap, uint64_t *out_len, const uint8_t *pre_key,
                           const uint8_t *pre_eph) {
    StagePool &pool = StagePool::get();
    if (!ecies_par_eligible(n) || !pool.try_acquire())
        return ecies_decrypt_snap(secret, secret_len, in, n, out, cap, out_len, nullptr, pre_key, pre_eph);
    struct Hold {  // the pool until every return below
        StagePool &p;
        ~Hold() { p.release(); }
    } hold{pool};
    const uint64_t m = n - ECIES_OVERHEAD;
    uint8_t key[32];
    if (pre_key && pre_eph && std::memcmp(pre_eph, in, 65) == 0) {
        std::memcpy(key, pre_key, 32);
    } else {
        const int st = ecies_derive_key(secret, secret_len, in, key);
        if (st != CHIP_OK) return st;
    }
    const uint8_t *iv = in + 65, *tag = in + 81, *ct = in + 97;
    Gcm msg;
    msg.init(key, iv, 16, false);
    OPENSSL_cleanse(key, 32);
    // 1: the ciphertext in 16-B aligned pieces on the pool's threads into a
    // plaintext buffer; the joined GHASH's tag checked first
    static thread_local std::vector<uint8_t> t_plain;
    if (t_plain.size() < m) t_plain.resize(m);
    ScratchCap cap_plain{t_plain};  // every return below wipes it first
    uint8_t *P = t_plain.data();
    const bool parts_ok = gcm_parts(pool, msg, ct, P, m);
    auto wipe_plain = [&] { wipe_parts(pool, P, m); };
    uint8_t t[16];
    msg.tag_joined(m, t);
    msg.wipe();
    const bool tag_ok = parts_ok && CRYPTO_memcmp(t, tag, 16) == 0;
    if (!tag_ok) {
        wipe_plain();
        return CHIP_ERR_ECIES;
    }
    // 2, 3: the frame stream's chunk headers walked, the chunks decoded on every thread
    const int st = snap_frames_par(pool, P, m, out, cap, out_len);
    wipe_plain();
    return st;
}

int ecies_encrypt_par_plain(const uint8_t *pubkey, uint64_t pubkey_len, const uint8_t *eph_sk,
                            const uint8_t *nonce, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap,
                            uint64_t *out_len) {
    StagePool &pool = StagePool::get();
    if (n < STAGE_PAR_MIN || !out || cap < n + ECIES_OVERHEAD || !gcm_vaes_on() || n > GCM_MAX_BYTES ||
        !pool.try_acquire())
        return ecies_encrypt(pubkey, pubkey_len, eph_sk, nonce, in, n, out, cap, out_len);
    struct Hold {
        StagePool &p;
        ~Hold() { p.release(); }
    } hold{pool};
    uint8_t peer[65];
    EciesKey key;
    int st = ecies_peer(pubkey, pubkey_len, peer);
    // k·G here and k·P on one of the held pool's workers (ecies_prepare's own
    // par_for would find the pool taken and run them one after the other)
    if (st == CHIP_OK)
        st = ecies_prepare_with(peer, eph_sk, &key, [&](const std::function<void(int)> &f) {
            pool.start([&](int w) {
                if (w == 1) f(1);
            });
            f(0);
            pool.wait();
        });
    uint8_t *iv = out + 65;
    if (st == CHIP_OK) {
        std::memcpy(out, key.eph_pub, 65);
        if (nonce) std::memcpy(iv, nonce, 16);
        else if (RAND_bytes(iv, 16) != 1) st = CHIP_ERR_ECIES;
    }
    if (st != CHIP_OK) {
        ecies_key_wipe(&key);
        return st;
    }
    Gcm msg;
    msg.init(key.key, iv, 16, true);
    ecies_key_wipe(&key);
    const bool parts_ok = gcm_parts(pool, msg, in, out + 97, n);
    msg.tag_joined(n, out + 81);
    msg.wipe();
    if (!parts_ok) return CHIP_ERR_ECIES;
    *out_len = n + ECIES_OVERHEAD;
    return CHIP_OK;
}

int ecies_decrypt_par(const uint8_t *secret, uint64_t secret_len, const uint8_t *in, uint64_t n, uint8_t *out,
                      uint64_t cap, uint64_t *out_len, const uint8_t *pre_key, const uint8_t *pre_eph) {
    StagePool &pool = StagePool::get();
    if (!ecies_par_eligible(n) || !out || cap < n - ECIES_OVERHEAD || !pool.try_acquire())
        return ecies_decrypt(secret, secret_len, in, n, out, cap, out_len, pre_key, pre_eph);
    struct Hold {
        StagePool &p;
        ~Hold() { p.release(); }
    } hold{pool};
    const uint64_t m = n - ECIES_OVERHEAD;
    uint8_t key[32];
    if (pre_key && pre_eph && std::memcmp(pre_eph, in, 65) == 0) {
        std::memcpy(key, pre_key, 32);
    } else {
        const int st = ecies_derive_key(secret, secret_len, in, key);
        if (st != CHIP_OK) return st;
    }
    Gcm msg;
    msg.init(key, in + 65, 16, false);
    OPENSSL_cleanse(key, 32);
    const bool parts_ok = gcm_parts(pool, msg, in + 97, out, m);
    uint8_t t[16];
    msg.tag_joined(m, t);
    msg.wipe();
    if (!parts_ok || CRYPTO_memcmp(t, in + 81, 16) != 0) {
        wipe_parts(pool, out, m);  // never hand back unauthenticated plaintext
        return CHIP_ERR_ECIES;
    }
    *out_len = m;
    return CHIP_OK;
}
}  // namespace host
}  // namespace chip
