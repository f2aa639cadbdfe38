// host_snap.cpp — snappy framing and CRC-32C for the host side of
// encode()/decode() (encoding.rs:16-28 `snap`; decoding.rs:62-77).
//
// Snappy: the framing format of snap 1.1.0's FrameEncoder — stream identifier,
// then one chunk per 64 KiB block: masked CRC-32C of the block, the block
// compressed, or stored raw when compression saves less than 1/8 (the
// `compress_len >= len - len/8` rule).  The block compressor restates the
// published snappy encodeBlock (Go snappy; snap 1.x is a port of it): hash
// table of 2^8..2^14 u16 entries, hash (u32 * 0x1E35A7BD) >> shift, the
// skip/32 search acceleration, 15-byte input margin, copies split 64/60 and
// encoded as copy-1 when len < 12 and offset < 2048.  Output for incompressible
// data is canonical (raw chunks); for compressible data it follows the
// restated algorithm (parity vs the snap crate itself is unpinned — DESIGN.md).
// The one-pass ECIES paths (host_stages.cpp) use the pieces in snap_internal.hpp.
#include "host_stages.hpp"
#include "snap_internal.hpp"

#include <immintrin.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/carbonado_hip.h"

namespace chip {
namespace host {

// ---------------------------------------------------------------- CRC-32C
// crc32q has a 3-cycle latency and issues every cycle, so one chain runs at a
// third of the instruction's rate.  Three chains over consecutive segments of
// B bytes, joined by the "append B zero bytes" map of the CRC register (a
// linear map over GF(2)^32, applied through four 256-entry tables):
// crc(c, X || Y) = zeros_|Y|(crc(c, X)) ^ crc(0, Y).  (A round-1 three-chain
// version measured slower end to end on a different decode pipeline, r1u;
// CHIP_CRC_CHAINS=1 keeps the one-chain form for the A/B.)
namespace {

__attribute__((target("sse4.2"))) inline uint32_t crc_raw1(uint32_t c32, const uint8_t *p, size_t n) {
    uint64_t c = c32;
    while (n >= 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c = _mm_crc32_u64(c, v);
        p += 8;
        n -= 8;
    }
    c32 = (uint32_t)c;
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return c32;
}

// the register after B zero bytes, as tables over its four bytes
struct CrcShift {
    uint32_t t[4][256];
    explicit CrcShift(size_t B) {
        std::vector<uint8_t> z(B, 0);
        uint32_t col[32];
        for (int i = 0; i < 32; ++i) col[i] = crc_raw1(1u << i, z.data(), B);
        for (int k = 0; k < 4; ++k)
            for (int b = 0; b < 256; ++b) {
                uint32_t x = 0;
                for (int j = 0; j < 8; ++j)
                    if (b >> j & 1) x ^= col[8 * k + j];
                t[k][b] = x;
            }
    }
    uint32_t operator()(uint32_t c) const {
        return t[0][c & 255] ^ t[1][(c >> 8) & 255] ^ t[2][(c >> 16) & 255] ^ t[3][c >> 24];
    }
};

// three chains over [p, p + 3B) in rounds; returns the register after them
template <size_t B>
__attribute__((target("sse4.2"))) inline uint32_t crc_raw3(uint32_t c0, const uint8_t *&p, size_t &n,
                                                           const CrcShift &sh) {
    while (n >= 3 * B) {
        uint64_t a = c0, b = 0, c = 0;
        for (size_t i = 0; i < B; i += 8) {
            uint64_t x, y, z;
            std::memcpy(&x, p + i, 8);
            std::memcpy(&y, p + B + i, 8);
            std::memcpy(&z, p + 2 * B + i, 8);
            a = _mm_crc32_u64(a, x);
            b = _mm_crc32_u64(b, y);
            c = _mm_crc32_u64(c, z);
        }
        c0 = sh(sh((uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)c;
        p += 3 * B;
        n -= 3 * B;
    }
    return c0;
}

bool crc_chains3() {
    static const bool on = [] {
        const char *v = std::getenv("CHIP_CRC_CHAINS");
        return !(v && v[0] == '1' && v[1] == 0);
    }();
    return on;
}

}  // namespace

uint32_t crc32c(const uint8_t *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    if (crc_chains3()) {
        static const CrcShift s4k(4096), s256(256);
        c = crc_raw3<4096>(c, p, n, s4k);
        c = crc_raw3<256>(c, p, n, s256);
    }
    return crc_raw1(c, p, n) ^ 0xFFFFFFFFu;
}

uint32_t crc_masked(const uint8_t *p, size_t n) {
    const uint32_t c = crc32c(p, n);
    return ((c >> 15) | (c << 17)) + 0xA282EAD8u;
}

// ---------------------------------------------------------------- snappy block
namespace {

constexpr size_t INPUT_MARGIN = 15;
constexpr size_t MIN_NON_LITERAL_BLOCK = 1 + 1 + INPUT_MARGIN;

inline uint32_t load32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline uint64_t load64(const uint8_t *p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

size_t put_varint(uint8_t *d, uint64_t v) {
    size_t i = 0;
    while (v >= 0x80) {
        d[i++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    d[i++] = (uint8_t)v;
    return i;
}

size_t emit_literal(uint8_t *d, const uint8_t *lit, size_t len) {
    const size_t n = len - 1;
    size_t i;
    if (n < 60) {
        d[0] = (uint8_t)(n << 2);
        i = 1;
    } else if (n < 256) {
        d[0] = 60 << 2;
        d[1] = (uint8_t)n;
        i = 2;
    } else {
        d[0] = 61 << 2;
        d[1] = (uint8_t)n;
        d[2] = (uint8_t)(n >> 8);
        i = 3;
    }
    std::memcpy(d + i, lit, len);
    return i + len;
}

size_t emit_copy(uint8_t *d, size_t offset, size_t len) {
    size_t i = 0;
    while (len >= 68) {  // length-64 copy-2
        d[i] = (63 << 2) | 2;
        d[i + 1] = (uint8_t)offset;
        d[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        len -= 64;
    }
    if (len > 64) {  // length-60 copy-2, leaving 5..8 for a short copy
        d[i] = (59 << 2) | 2;
        d[i + 1] = (uint8_t)offset;
        d[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        len -= 60;
    }
    if (len >= 12 || offset >= 2048) {
        d[i] = (uint8_t)(((len - 1) << 2) | 2);
        d[i + 1] = (uint8_t)offset;
        d[i + 2] = (uint8_t)(offset >> 8);
        return i + 3;
    }
    d[i] = (uint8_t)(((offset >> 8) << 5) | ((len - 4) << 2) | 1);
    d[i + 1] = (uint8_t)offset;
    return i + 2;
}

// One block (n >= MIN_NON_LITERAL_BLOCK, n <= 64 KiB) without the varint header.
size_t encode_block(uint8_t *dst, const uint8_t *src, size_t n) {
    uint32_t shift = 24;
    size_t tsize = 256;
    while (tsize < 16384 && tsize < n) {
        --shift;
        tsize <<= 1;
    }
    uint16_t table[16384];
    std::memset(table, 0, tsize * sizeof(uint16_t));
    auto hash = [shift](uint32_t u) -> size_t { return (size_t)((u * 0x1E35A7BDu) >> shift); };

    const size_t s_limit = n - INPUT_MARGIN;
    size_t next_emit = 0, d = 0, s = 1;
    size_t next_hash = hash(load32(src + s));
    for (;;) {
        size_t skip = 32, s_next = s, cand;
        for (;;) {
            s = s_next;
            const size_t step = skip >> 5;
            s_next = s + step;
            skip += step;
            if (s_next > s_limit) goto remainder;
            cand = table[next_hash];
            table[next_hash] = (uint16_t)s;
            next_hash = hash(load32(src + s_next));
            if (load32(src + s) == load32(src + cand)) break;
        }
        d += emit_literal(dst + d, src + next_emit, s - next_emit);
        for (;;) {
            const size_t base = s;
            s += 4;
            // extend the match 8 bytes at a time (the first differing byte from
            // the XOR's trailing zeros), then bytewise at the block's end
            size_t i = cand + 4;
            for (;;) {
                if (s + 8 > n) {
                    while (s < n && src[i] == src[s]) ++i, ++s;
                    break;
                }
                const uint64_t x = load64(src + s) ^ load64(src + i);
                if (x) {
                    s += (size_t)__builtin_ctzll(x) >> 3;
                    break;
                }
                s += 8;
                i += 8;
            }
            d += emit_copy(dst + d, base - cand, s - base);
            next_emit = s;
            if (s >= s_limit) goto remainder;
            const uint64_t x = load64(src + s - 1);
            table[hash((uint32_t)x)] = (uint16_t)(s - 1);
            const size_t ch = hash((uint32_t)(x >> 8));
            cand = table[ch];
            table[ch] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != load32(src + cand)) {
                next_hash = hash((uint32_t)(x >> 16));
                ++s;
                break;
            }
        }
    }
remainder:
    if (next_emit < n) d += emit_literal(dst + d, src + next_emit, n - next_emit);
    return d;
}

// Raw snappy of one block (<= 64 KiB), varint header included.
size_t compress_raw(uint8_t *dst, const uint8_t *src, size_t n) {
    if (n == 0) {
        dst[0] = 0;
        return 1;
    }
    size_t d = put_varint(dst, n);
    if (n < MIN_NON_LITERAL_BLOCK) return d + emit_literal(dst + d, src, n);
    return d + encode_block(dst + d, src, n);
}

}  // namespace

bool get_varint(const uint8_t *p, size_t n, uint64_t *v, size_t *used) {
    uint64_t r = 0;
    for (size_t i = 0; i < n && i < 10; ++i) {
        r |= (uint64_t)(p[i] & 0x7F) << (7 * i);
        if (!(p[i] & 0x80)) {
            *v = r;
            *used = i + 1;
            return true;
        }
    }
    return false;
}

// Raw snappy block decode into out[0..cap); returns false on corrupt input.
bool decompress_raw(const uint8_t *src, size_t n, uint8_t *out, size_t cap, size_t *out_len) {
    uint64_t dlen;
    size_t used;
    if (!get_varint(src, n, &dlen, &used) || dlen > cap) return false;
    size_t s = used, d = 0;
    while (s < n) {
        const uint8_t tag = src[s];
        size_t len, off;
        switch (tag & 3) {
            case 0: {  // literal
                size_t x = tag >> 2;
                if (x < 60) {
                    s += 1;
                } else {
                    const size_t nb = x - 59;  // 1..4 length bytes
                    if (s + 1 + nb > n) return false;
                    x = 0;
                    for (size_t b = 0; b < nb; ++b) x |= (size_t)src[s + 1 + b] << (8 * b);
                    s += 1 + nb;
                }
                len = x + 1;
                if (len > n - s || len > dlen - d) return false;
                std::memcpy(out + d, src + s, len);
                s += len;
                d += len;
                continue;
            }
            case 1:
                if (s + 2 > n) return false;
                len = 4 + ((tag >> 2) & 7);
                off = ((size_t)(tag >> 5) << 8) | src[s + 1];
                s += 2;
                break;
            case 2:
                if (s + 3 > n) return false;
                len = 1 + (tag >> 2);
                off = (size_t)src[s + 1] | ((size_t)src[s + 2] << 8);
                s += 3;
                break;
            default:
                if (s + 5 > n) return false;
                len = 1 + (tag >> 2);
                off = (size_t)load32(src + s + 1);
                s += 5;
                break;
        }
        if (off == 0 || off > d || len > dlen - d) return false;
        uint8_t *dp = out + d;
        const uint8_t *sp = dp - off;
        if (off >= len) {  // source and destination apart
            std::memcpy(dp, sp, len);
        } else if (off >= 8) {  // 8-B pieces, each from bytes already written
            size_t i = 0;
            for (; i + 8 <= len; i += 8) std::memcpy(dp + i, sp + i, 8);
            for (; i < len; ++i) dp[i] = sp[i];
        } else {  // a pattern shorter than 8 bytes repeated: byte by byte
            for (size_t i = 0; i < len; ++i) dp[i] = sp[i];
        }
        d += len;
    }
    if (d != dlen) return false;
    *out_len = d;
    return true;
}

uint64_t snap_max_len(uint64_t n) {
    if (n == 0) return 0;
    return sizeof(STREAM_ID) + 8 * ((n + MAX_BLOCK - 1) / MAX_BLOCK) + n;
}

// One chunk of the frame stream for len (<= MAX_BLOCK) input bytes: its 8-B
// header into hdr, its body (compressed into tmp, or the input itself when
// compression saves less than 1/8: FrameEncoder's rule) at *body.
size_t snap_block(const uint8_t *src, size_t len, uint8_t hdr[8], uint8_t *tmp, const uint8_t **body) {
    const uint32_t crc = crc_masked(src, len);
    const size_t clen = compress_raw(tmp, src, len);
    const bool raw = clen >= len - len / 8;
    const size_t blen = raw ? len : clen;
    const uint32_t chunk_len = (uint32_t)(4 + blen);
    hdr[0] = raw ? 0x01 : 0x00;
    hdr[1] = (uint8_t)chunk_len;
    hdr[2] = (uint8_t)(chunk_len >> 8);
    hdr[3] = (uint8_t)(chunk_len >> 16);
    std::memcpy(hdr + 4, &crc, 4);
    *body = raw ? src : tmp;
    return blen;
}

int snap_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    // FrameEncoder writes nothing at all for an empty input (no stream id).
    if (n == 0) {
        *out_len = 0;
        return CHIP_OK;
    }
    if (cap < snap_max_len(n)) return CHIP_ERR_BUFFER_TOO_SMALL;
    std::vector<uint8_t> tmp(MAX_COMPRESS_BLOCK);
    uint64_t d = 0;
    std::memcpy(out, STREAM_ID, sizeof(STREAM_ID));
    d += sizeof(STREAM_ID);
    for (uint64_t o = 0; o < n; o += MAX_BLOCK) {
        const size_t len = (size_t)((n - o) < MAX_BLOCK ? (n - o) : MAX_BLOCK);
        const uint8_t *body;
        const size_t blen = snap_block(in + o, len, out + d, tmp.data(), &body);
        std::memcpy(out + d + 8, body, blen);
        d += 8 + blen;
    }
    *out_len = d;
    return CHIP_OK;
}

// Walk the chunks; if `out` is null only sizes are computed.
static int snap_walk(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    uint64_t s = 0, d = 0;
    bool ident = false;
    while (s < n) {
        if (n - s < 4) return CHIP_ERR_SNAP;
        const uint8_t ty = in[s];
        const uint64_t clen = (uint64_t)in[s + 1] | ((uint64_t)in[s + 2] << 8) | ((uint64_t)in[s + 3] << 16);
        s += 4;
        if (clen > n - s) return CHIP_ERR_SNAP;
        const uint8_t *body = in + s;
        if (!ident && ty != 0xFF) return CHIP_ERR_SNAP;  // stream must open with the identifier
        if (ty == 0xFF) {
            if (clen != 6 || std::memcmp(body, STREAM_ID + 4, 6) != 0) return CHIP_ERR_SNAP;
            ident = true;
        } else if (ty == 0x00 || ty == 0x01) {
            if (clen < 4) return CHIP_ERR_SNAP;
            uint32_t want;
            std::memcpy(&want, body, 4);
            const uint8_t *data = body + 4;
            const uint64_t dl = clen - 4;
            if (ty == 0x01) {
                if (dl > MAX_BLOCK) return CHIP_ERR_SNAP;
                if (out) {
                    if (dl > cap - d) return CHIP_ERR_BUFFER_TOO_SMALL;
                    if (crc_masked(data, dl) != want) return CHIP_ERR_SNAP;
                    std::memcpy(out + d, data, dl);
                }
                d += dl;
            } else {
                uint64_t ulen;
                size_t used;
                if (!get_varint(data, dl, &ulen, &used) || ulen > MAX_BLOCK) return CHIP_ERR_SNAP;
                if (out) {
                    if (ulen > cap - d) return CHIP_ERR_BUFFER_TOO_SMALL;
                    size_t got;
                    if (!decompress_raw(data, dl, out + d, ulen, &got) || got != ulen) return CHIP_ERR_SNAP;
                    if (crc_masked(out + d, ulen) != want) return CHIP_ERR_SNAP;
                }
                d += ulen;
            }
        } else if (ty >= 0x02 && ty <= 0x7F) {
            return CHIP_ERR_SNAP;  // reserved unskippable
        }  // 0x80..0xFE: padding / reserved skippable
        s += clen;
    }
    *out_len = d;
    return CHIP_OK;
}

int snap_decompressed_len(const uint8_t *in, uint64_t n, uint64_t *len) {
    return snap_walk(in, n, nullptr, 0, len);
}

int snap_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    uint64_t need;
    int st = snap_walk(in, n, nullptr, 0, &need);
    if (st != CHIP_OK) return st;
    if (need > cap || (need && !out)) {
        *out_len = need;
        return CHIP_ERR_BUFFER_TOO_SMALL;
    }
    return snap_walk(in, n, out, cap, out_len);
}

}  // namespace host
}  // namespace chip
