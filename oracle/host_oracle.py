"""Pure-Python restatement of the host stages of encode()/decode() —
TEST INFRASTRUCTURE ONLY (never imported by the product).

Covers the stages the reference runs before zfec and after zfec-decode:
  * `encoding::snap` / `decoding::snap` (reference src/encoding.rs:16-28,
    src/decoding.rs:70-77) -> snap 1.1.0 FrameEncoder / FrameDecoder
    (third-party, absent from /root/reference): framing per the published
    snappy framing format; the block compressor restates the published snappy
    `encodeBlock` (Go snappy, which snap 1.x ports).
  * `encoding::ecies` / `decoding::ecies` (src/encoding.rs:30-36,
    src/decoding.rs:62-68) -> ecies 0.2.6 (third-party, absent) with its
    default config: secp256k1, uncompressed ephemeral and HKDF keys,
    HKDF-SHA256 (no salt, no info), AES-256-GCM with a 16-byte nonce,
    output eph_pub65 || nonce16 || tag16 || ciphertext.

Written independently of OpenSSL (which the product links): SHA-256
(FIPS 180-4), HMAC (RFC 2104), HKDF (RFC 5869), AES-256 (FIPS-197), GCM
(SP 800-38D) and secp256k1 affine arithmetic are all restated here and pinned
by published known answers in tests/golden/host_kat.json.

Parity status: the primitives are pinned by published vectors; the snappy
bytes of incompressible blocks are canonical (stored raw); the compressed
form of compressible blocks and the exact ecies composition follow the
restated algorithms and are NOT pinned by the reference crates themselves
(neither is buildable here) — see DESIGN.md "Oracle".
"""
from __future__ import annotations

import struct

# ---------------------------------------------------------------- SHA-256
_K256 = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
]
M32 = 0xFFFFFFFF


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def sha256(data: bytes) -> bytes:
    h = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
    ml = len(data) * 8
    data = data + b"\x80" + b"\0" * ((55 - len(data)) % 64) + struct.pack(">Q", ml)
    for o in range(0, len(data), 64):
        w = list(struct.unpack(">16I", data[o:o + 64]))
        for i in range(16, 64):
            s0 = _rotr(w[i - 15], 7) ^ _rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
            s1 = _rotr(w[i - 2], 17) ^ _rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
            w.append((w[i - 16] + s0 + w[i - 7] + s1) & M32)
        a, b, c, d, e, f, g, hh = h
        for i in range(64):
            t1 = (hh + (_rotr(e, 6) ^ _rotr(e, 11) ^ _rotr(e, 25)) + ((e & f) ^ (~e & g)) + _K256[i] + w[i]) & M32
            t2 = ((_rotr(a, 2) ^ _rotr(a, 13) ^ _rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M32
            hh, g, f, e, d, c, b, a = g, f, e, (d + t1) & M32, c, b, a, (t1 + t2) & M32
        h = [(x + y) & M32 for x, y in zip(h, [a, b, c, d, e, f, g, hh])]
    return struct.pack(">8I", *h)


def hmac_sha256(key: bytes, msg: bytes) -> bytes:
    if len(key) > 64:
        key = sha256(key)
    key = key + b"\0" * (64 - len(key))
    return sha256(bytes(k ^ 0x5C for k in key) + sha256(bytes(k ^ 0x36 for k in key) + msg))


def hkdf_sha256(ikm: bytes, salt: bytes | None = None, info: bytes = b"", length: int = 32) -> bytes:
    prk = hmac_sha256(salt if salt else b"\0" * 32, ikm)
    okm, t, i = b"", b"", 1
    while len(okm) < length:
        t = hmac_sha256(prk, t + info + bytes([i]))
        okm += t
        i += 1
    return okm[:length]


# ---------------------------------------------------------------- AES-256
def _xtime(a):
    return ((a << 1) ^ 0x1B) & 0xFF if a & 0x80 else a << 1


def _gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xtime(a)
        b >>= 1
    return r


def _make_sbox():
    sbox = [0] * 256
    for x in range(256):
        inv = 0 if x == 0 else next(y for y in range(1, 256) if _gmul(x, y) == 1)
        s = inv
        for r in (1, 2, 3, 4):
            s ^= ((inv << r) | (inv >> (8 - r))) & 0xFF
        sbox[x] = s ^ 0x63
    return sbox


SBOX = _make_sbox()
# T-table: column contribution of S[x] through MixColumns, as a 32-bit word
_T0 = [(_gmul(s, 2) << 24) | (s << 16) | (s << 8) | _gmul(s, 3) for s in SBOX]
_T1 = [((t >> 8) | (t << 24)) & M32 for t in _T0]
_T2 = [((t >> 16) | (t << 16)) & M32 for t in _T0]
_T3 = [((t >> 24) | (t << 8)) & M32 for t in _T0]


def aes256_expand(key: bytes) -> list[int]:
    assert len(key) == 32
    w = list(struct.unpack(">8I", key))
    rcon = 1
    for i in range(8, 60):
        t = w[i - 1]
        if i % 8 == 0:
            t = ((t << 8) | (t >> 24)) & M32
            t = (SBOX[t >> 24] << 24) | (SBOX[(t >> 16) & 0xFF] << 16) | (SBOX[(t >> 8) & 0xFF] << 8) | SBOX[t & 0xFF]
            t ^= rcon << 24
            rcon = _xtime(rcon)
        elif i % 8 == 4:
            t = (SBOX[t >> 24] << 24) | (SBOX[(t >> 16) & 0xFF] << 16) | (SBOX[(t >> 8) & 0xFF] << 8) | SBOX[t & 0xFF]
        w.append(w[i - 8] ^ t)
    return w


def aes256_block(rk: list[int], block: bytes) -> bytes:
    s0, s1, s2, s3 = struct.unpack(">4I", block)
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3]
    for r in range(1, 14):
        k = 4 * r
        t0 = _T0[s0 >> 24] ^ _T1[(s1 >> 16) & 0xFF] ^ _T2[(s2 >> 8) & 0xFF] ^ _T3[s3 & 0xFF] ^ rk[k]
        t1 = _T0[s1 >> 24] ^ _T1[(s2 >> 16) & 0xFF] ^ _T2[(s3 >> 8) & 0xFF] ^ _T3[s0 & 0xFF] ^ rk[k + 1]
        t2 = _T0[s2 >> 24] ^ _T1[(s3 >> 16) & 0xFF] ^ _T2[(s0 >> 8) & 0xFF] ^ _T3[s1 & 0xFF] ^ rk[k + 2]
        t3 = _T0[s3 >> 24] ^ _T1[(s0 >> 16) & 0xFF] ^ _T2[(s1 >> 8) & 0xFF] ^ _T3[s2 & 0xFF] ^ rk[k + 3]
        s0, s1, s2, s3 = t0, t1, t2, t3

    def last(a, b, c, d, k):
        return ((SBOX[a >> 24] << 24) | (SBOX[(b >> 16) & 0xFF] << 16) | (SBOX[(c >> 8) & 0xFF] << 8)
                | SBOX[d & 0xFF]) ^ k

    return struct.pack(">4I", last(s0, s1, s2, s3, rk[56]), last(s1, s2, s3, s0, rk[57]),
                       last(s2, s3, s0, s1, rk[58]), last(s3, s0, s1, s2, rk[59]))


# ---------------------------------------------------------------- GCM
_R = 0xE1 << 120


def _gf128_mul(x: int, y: int) -> int:
    """SP 800-38D Algorithm 1 (bit-reflected GF(2^128))."""
    z, v = 0, y
    for i in range(127, -1, -1):
        if (x >> i) & 1:
            z ^= v
        v = (v >> 1) ^ _R if v & 1 else v >> 1
    return z


def _ghash(h: int, data: bytes) -> int:
    y = 0
    for o in range(0, len(data), 16):
        y = _gf128_mul(y ^ int.from_bytes(data[o:o + 16], "big"), h)
    return y


def _pad16(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 16)


def _gctr(rk, icb: int, data: bytes) -> bytes:
    out = bytearray()
    cb = icb
    for o in range(0, len(data), 16):
        ks = aes256_block(rk, cb.to_bytes(16, "big"))
        blk = data[o:o + 16]
        out += bytes(a ^ b for a, b in zip(blk, ks))
        cb = (cb & ~M32) | ((cb + 1) & M32)  # inc32
    return bytes(out)


def aes256_gcm_encrypt(key: bytes, iv: bytes, pt: bytes, aad: bytes = b"") -> tuple[bytes, bytes]:
    rk = aes256_expand(key)
    h = int.from_bytes(aes256_block(rk, b"\0" * 16), "big")
    if len(iv) == 12:
        j0 = int.from_bytes(iv + b"\0\0\0\1", "big")
    else:
        j0 = _ghash(h, _pad16(iv) + b"\0" * 8 + struct.pack(">Q", len(iv) * 8))
    ct = _gctr(rk, (j0 & ~M32) | ((j0 + 1) & M32), pt)
    s = _ghash(h, _pad16(aad) + _pad16(ct) + struct.pack(">QQ", len(aad) * 8, len(ct) * 8))
    tag = _gctr(rk, j0, s.to_bytes(16, "big"))
    return ct, tag


def aes256_gcm_decrypt(key: bytes, iv: bytes, ct: bytes, tag: bytes, aad: bytes = b"") -> bytes | None:
    rk = aes256_expand(key)
    h = int.from_bytes(aes256_block(rk, b"\0" * 16), "big")
    if len(iv) == 12:
        j0 = int.from_bytes(iv + b"\0\0\0\1", "big")
    else:
        j0 = _ghash(h, _pad16(iv) + b"\0" * 8 + struct.pack(">Q", len(iv) * 8))
    s = _ghash(h, _pad16(aad) + _pad16(ct) + struct.pack(">QQ", len(aad) * 8, len(ct) * 8))
    if _gctr(rk, j0, s.to_bytes(16, "big")) != tag:
        return None
    return _gctr(rk, (j0 & ~M32) | ((j0 + 1) & M32), ct)


# ---------------------------------------------------------------- secp256k1
P = 2 ** 256 - 2 ** 32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def on_curve(pt) -> bool:
    x, y = pt
    return (y * y - x * x * x - 7) % P == 0


def _add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def point_mul(k: int, pt=(GX, GY)):
    r = None
    while k:
        if k & 1:
            r = _add(r, pt)
        pt = _add(pt, pt)
        k >>= 1
    return r


def ser_uncompressed(pt) -> bytes:
    return b"\x04" + pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


def parse_pubkey(b: bytes):
    """libsecp256k1 PublicKey::parse_slice(.., None): 33, 64 or 65 bytes."""
    if len(b) == 64:
        b = b"\x04" + b
    if len(b) == 65 and b[0] == 4:
        pt = (int.from_bytes(b[1:33], "big"), int.from_bytes(b[33:], "big"))
    elif len(b) == 33 and b[0] in (2, 3):
        x = int.from_bytes(b[1:], "big")
        y = pow((x ** 3 + 7) % P, (P + 1) // 4, P)
        if (y & 1) != (b[0] & 1):
            y = P - y
        pt = (x, y)
    else:
        raise ValueError("bad public key")
    if not (pt[0] < P and pt[1] < P and on_curve(pt)):
        raise ValueError("point not on curve")
    return pt


def public_key(sk: bytes) -> bytes:
    k = int.from_bytes(sk, "big")
    assert 0 < k < N
    return ser_uncompressed(point_mul(k))


def ecies_encrypt(receiver_pub: bytes, msg: bytes, eph_sk: bytes, nonce: bytes) -> bytes:
    """ecies 0.2.6 encrypt with injected ephemeral key and nonce."""
    peer = parse_pubkey(receiver_pub)
    k = int.from_bytes(eph_sk, "big")
    assert 0 < k < N and len(nonce) == 16
    eph_pub = ser_uncompressed(point_mul(k))
    shared = ser_uncompressed(point_mul(k, peer))
    key = hkdf_sha256(eph_pub + shared)
    ct, tag = aes256_gcm_encrypt(key, nonce, msg)
    return eph_pub + nonce + tag + ct


def ecies_decrypt(sk: bytes, data: bytes) -> bytes:
    k = int.from_bytes(sk, "big")
    if len(sk) != 32 or not 0 < k < N or len(data) < 97:
        raise ValueError("ecies error")
    eph = parse_pubkey(data[:65])
    shared = ser_uncompressed(point_mul(k, eph))
    key = hkdf_sha256(data[:65] + shared)
    pt = aes256_gcm_decrypt(key, data[65:81], data[97:], data[81:97])
    if pt is None:
        raise ValueError("ecies error")
    return pt


# ---------------------------------------------------------------- CRC-32C
def _crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_CRC = _crc_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def crc32c_masked(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & M32


# ---------------------------------------------------------------- snappy
MAX_BLOCK = 65536
INPUT_MARGIN = 15
STREAM_ID = b"\xff\x06\x00\x00sNaPpY"


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _lit(lit: bytes) -> bytes:
    n = len(lit) - 1
    if n < 60:
        return bytes([n << 2]) + lit
    if n < 256:
        return bytes([60 << 2, n]) + lit
    return bytes([61 << 2, n & 0xFF, n >> 8]) + lit


def _copy(offset: int, length: int) -> bytes:
    out = bytearray()
    while length >= 68:
        out += bytes([(63 << 2) | 2, offset & 0xFF, offset >> 8])
        length -= 64
    if length > 64:
        out += bytes([(59 << 2) | 2, offset & 0xFF, offset >> 8])
        length -= 60
    if length >= 12 or offset >= 2048:
        out += bytes([((length - 1) << 2) | 2, offset & 0xFF, offset >> 8])
    else:
        out += bytes([((offset >> 8) << 5) | ((length - 4) << 2) | 1, offset & 0xFF])
    return bytes(out)


def _u32(b: bytes, i: int) -> int:
    return int.from_bytes(b[i:i + 4], "little")


def snappy_block(src: bytes) -> bytes:
    """Raw snappy of one block (<= 64 KiB) incl. the varint length."""
    n = len(src)
    if n == 0:
        return b"\x00"
    out = bytearray(_varint(n))
    if n < 1 + 1 + INPUT_MARGIN:
        return bytes(out + _lit(src))
    shift, tsize = 24, 256
    while tsize < 16384 and tsize < n:
        shift -= 1
        tsize *= 2
    table = [0] * tsize

    def h(u):
        return ((u * 0x1E35A7BD) & M32) >> shift

    s_limit = n - INPUT_MARGIN
    next_emit, s = 0, 1
    next_hash = h(_u32(src, s))
    while True:
        skip, s_next = 32, s
        while True:
            s = s_next
            step = skip >> 5
            s_next = s + step
            skip += step
            if s_next > s_limit:
                if next_emit < n:
                    out += _lit(src[next_emit:])
                return bytes(out)
            cand = table[next_hash]
            table[next_hash] = s
            next_hash = h(_u32(src, s_next))
            if src[s:s + 4] == src[cand:cand + 4]:
                break
        out += _lit(src[next_emit:s])
        while True:
            base = s
            s += 4
            i = cand + 4
            while s < n and src[i] == src[s]:
                i += 1
                s += 1
            out += _copy(base - cand, s - base)
            next_emit = s
            if s >= s_limit:
                if next_emit < n:
                    out += _lit(src[next_emit:])
                return bytes(out)
            table[h(_u32(src, s - 1))] = s - 1
            ch = h(_u32(src, s))
            cand = table[ch]
            table[ch] = s
            if src[s:s + 4] != src[cand:cand + 4]:
                next_hash = h(_u32(src, s + 1))
                s += 1
                break


def snap_compress(data: bytes) -> bytes:
    """snap::write::FrameEncoder + write_all + into_inner (encoding.rs:17-27)."""
    if not data:
        return b""
    out = bytearray(STREAM_ID)
    for o in range(0, len(data), MAX_BLOCK):
        blk = data[o:o + MAX_BLOCK]
        crc = crc32c_masked(blk)
        comp = snappy_block(blk)
        raw = len(comp) >= len(blk) - len(blk) // 8
        body = blk if raw else comp
        out += bytes([1 if raw else 0]) + (4 + len(body)).to_bytes(3, "little") + struct.pack("<I", crc) + body
    return bytes(out)


def snappy_unblock(src: bytes) -> bytes:
    n, i, shift = 0, 0, 0
    while True:
        b = src[i]
        n |= (b & 0x7F) << shift
        i += 1
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while i < len(src):
        tag = src[i]
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln < 60:
                i += 1
            else:
                nb = ln - 59
                ln = int.from_bytes(src[i + 1:i + 1 + nb], "little")
                i += 1 + nb
            ln += 1
            out += src[i:i + ln]
            i += ln
            continue
        if kind == 1:
            ln = 4 + ((tag >> 2) & 7)
            off = ((tag >> 5) << 8) | src[i + 1]
            i += 2
        elif kind == 2:
            ln = 1 + (tag >> 2)
            off = int.from_bytes(src[i + 1:i + 3], "little")
            i += 3
        else:
            ln = 1 + (tag >> 2)
            off = int.from_bytes(src[i + 1:i + 5], "little")
            i += 5
        if off == 0 or off > len(out):
            raise ValueError("snappy: bad offset")
        for _ in range(ln):
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("snappy: length mismatch")
    return bytes(out)


def snap_decompress(data: bytes) -> bytes:
    """snap::read::FrameDecoder::read_to_end (decoding.rs:70-77)."""
    out = bytearray()
    i, ident = 0, False
    while i < len(data):
        if len(data) - i < 4:
            raise ValueError("snap: truncated chunk header")
        ty = data[i]
        ln = int.from_bytes(data[i + 1:i + 4], "little")
        body = data[i + 4:i + 4 + ln]
        if len(body) != ln:
            raise ValueError("snap: truncated chunk")
        if not ident and ty != 0xFF:
            raise ValueError("snap: missing stream identifier")
        if ty == 0xFF:
            if body != STREAM_ID[4:]:
                raise ValueError("snap: bad stream identifier")
            ident = True
        elif ty in (0, 1):
            crc = struct.unpack("<I", body[:4])[0]
            blk = body[4:] if ty == 1 else snappy_unblock(body[4:])
            if len(blk) > MAX_BLOCK or crc32c_masked(blk) != crc:
                raise ValueError("snap: checksum mismatch")
            out += blk
        elif 0x02 <= ty <= 0x7F:
            raise ValueError("snap: reserved unskippable chunk")
        i += 4 + ln
    return bytes(out)


# ---------------------------------------------------------------- pipeline
def host_encode(data: bytes, fmt: int, pubkey: bytes | None = None, eph_sk: bytes | None = None,
                nonce: bytes | None = None) -> tuple[bytes, int, int]:
    """encoding.rs:101-115: snap then ecies.  Returns (bytes entering zfec,
    bytes_compressed, bytes_encrypted)."""
    bc = be = 0
    cur = data
    if fmt & 2:
        cur = snap_compress(cur)
        bc = len(cur)
    if fmt & 1:
        cur = ecies_encrypt(pubkey, cur, eph_sk, nonce)
        be = len(cur)
    return cur, bc, be


def host_decode(data: bytes, fmt: int, secret: bytes | None = None) -> bytes:
    """decoding.rs:101-111: ecies then snap."""
    cur = data
    if fmt & 1:
        cur = ecies_decrypt(secret, cur)
    if fmt & 2:
        cur = snap_decompress(cur)
    return cur


# ---------------------------------------------------------------- BIP-340 + header
# The flat-file container (reference src/file.rs): Header::new signs the bao
# hash with secp256k1 0.28's Keypair::sign_schnorr (file.rs:263-289), i.e.
# BIP-340 with 32 bytes of auxiliary randomness from thread_rng; parsing
# verifies it against the x-only key of the stored pubkey (file.rs:129-131).
# Restated from the BIP-340 specification (tagged hashes, even-y keys and
# nonces), pinned by its published test vectors in tests/golden/host_kat.json.
MAGICNO = b"CARBONADO01\n"  # constants.rs:4
HEADER_LEN = 160            # file.rs:257-259


def tagged_hash(tag: str, msg: bytes) -> bytes:
    th = sha256(tag.encode())
    return sha256(th + th + msg)


def _lift_x(x: int):
    if x >= P:
        return None
    c = (pow(x, 3, P) + 7) % P
    y = pow(c, (P + 1) // 4, P)
    if y * y % P != c:
        return None
    return x, (y if y % 2 == 0 else P - y)


def schnorr_sign(sk: bytes, msg: bytes, aux: bytes) -> bytes:
    d0 = int.from_bytes(sk, "big")
    if len(sk) != 32 or not 0 < d0 < N or len(aux) != 32:
        raise ValueError("bad secret key")
    pub = point_mul(d0)
    d = d0 if pub[1] % 2 == 0 else N - d0
    t = bytes(a ^ b for a, b in zip(d.to_bytes(32, "big"), tagged_hash("BIP0340/aux", aux)))
    px = pub[0].to_bytes(32, "big")
    k0 = int.from_bytes(tagged_hash("BIP0340/nonce", t + px + msg), "big") % N
    if k0 == 0:
        raise ValueError("nonce is zero")
    r = point_mul(k0)
    k = k0 if r[1] % 2 == 0 else N - k0
    rx = r[0].to_bytes(32, "big")
    e = int.from_bytes(tagged_hash("BIP0340/challenge", rx + px + msg), "big") % N
    return rx + ((k + e * d) % N).to_bytes(32, "big")


def schnorr_verify(pkx: bytes, msg: bytes, sig: bytes) -> bool:
    pt = _lift_x(int.from_bytes(pkx, "big"))
    if pt is None or len(sig) != 64:
        return False
    r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big")
    if r >= P or s >= N:
        return False
    e = int.from_bytes(tagged_hash("BIP0340/challenge", sig[:32] + pkx + msg), "big") % N
    big_r = _add(point_mul(s), point_mul(N - e, pt) if e else None)
    return big_r is not None and big_r[1] % 2 == 0 and big_r[0] == r


def ser_compressed(pt) -> bytes:
    return bytes([2 + (pt[1] & 1)]) + pt[0].to_bytes(32, "big")


def header_bytes(sk: bytes, pk: bytes, hash32: bytes, fmt: int, chunk_index: int, encoded_len: int,
                 padding_len: int, metadata: bytes | None, aux: bytes) -> bytes:
    """Header::new + Header::try_to_vec (file.rs:263-335)."""
    if len(hash32) != 32:
        raise ValueError("message must be 32 bytes")
    pub = parse_pubkey(pk)
    sig = schnorr_sign(sk, hash32, aux)
    out = (MAGICNO + ser_compressed(pub) + hash32 + sig + bytes([fmt, chunk_index]) +
           encoded_len.to_bytes(4, "little") + padding_len.to_bytes(4, "little") +
           (metadata if metadata is not None else bytes(8)) + b"\x00")
    assert len(out) == HEADER_LEN
    return out


def header_parse(b: bytes) -> dict:
    """Header::try_from(&[u8]) (file.rs:116-154): magic, pubkey, signature."""
    if len(b) < HEADER_LEN - 1:
        raise ValueError("InvalidHeaderLength")
    if b[:12] != MAGICNO:
        raise ValueError("InvalidMagicNumber")
    pub = parse_pubkey(b[12:45])
    h, sig = b[45:77], b[77:141]
    if not schnorr_verify(pub[0].to_bytes(32, "big"), h, sig):
        raise ValueError("signature")
    meta = b[151:159]
    return {"pubkey": b[12:45], "hash": h, "signature": sig, "format": b[141], "chunk_index": b[142],
            "encoded_len": int.from_bytes(b[143:147], "little"), "padding_len": int.from_bytes(b[147:151], "little"),
            "metadata": meta if any(meta) else None}
