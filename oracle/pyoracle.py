"""Independent pure-Python restatement — TEST INFRASTRUCTURE ONLY.

A second, separately written oracle used to cross-check the C oracle
(carbonado_oracle.c) on small inputs.  It deliberately takes different
routes where the maths allows:
  * zfec enc_matrix via fec.c's own Vandermonde-specific inversion
    (`_invert_vdm`: coefficients of prod (x - p_i), synthetic division),
    where the C oracle uses generic Gauss-Jordan;
  * BLAKE3 via the spec's incremental "CV stack" (merge while the chunk
    count has trailing zero bits), where the C oracle recurses on the
    left-subtree-size rule;
  * bao layout by explicit pre-order recursion on node objects.
References: zfec fec.c (fec_new, _invert_vdm, generate_gf); BLAKE3 paper
section 2 and reference_impl.py; bao spec (combined encoding).
"""
from __future__ import annotations

import struct

# ---------------- GF(2^8) as in fec.c generate_gf() ----------------
PP = "101110001"  # x^8+x^4+x^3+x^2+1 read LSB first
GF_EXP = [0] * 510
GF_LOG = [0] * 256


def _generate_gf() -> None:
    mask = 1
    GF_EXP[8] = 0
    for i in range(8):
        GF_EXP[i] = mask
        GF_LOG[GF_EXP[i]] = i
        if PP[i] == "1":
            GF_EXP[8] ^= mask
        mask <<= 1
    GF_LOG[GF_EXP[8]] = 8
    mask = 1 << 7
    for i in range(9, 255):
        if GF_EXP[i - 1] >= mask:
            GF_EXP[i] = GF_EXP[8] ^ ((GF_EXP[i - 1] ^ mask) << 1)
        else:
            GF_EXP[i] = GF_EXP[i - 1] << 1
        GF_LOG[GF_EXP[i]] = i
    GF_LOG[0] = 255
    for i in range(255):
        GF_EXP[i + 255] = GF_EXP[i]


_generate_gf()
INVERSE = [0] * 256
for _i in range(1, 256):
    INVERSE[_i] = GF_EXP[255 - GF_LOG[_i]]


def gf_mul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return GF_EXP[GF_LOG[a] + GF_LOG[b]]


def _invert_vdm(src: list[int], k: int) -> None:
    """fec.c _invert_vdm: invert a Vandermonde matrix whose row i is the
    powers of p_i = src[i*k + 1]."""
    if k == 1:
        return
    c = [0] * k
    b = [0] * k
    p = [src[i * k + 1] for i in range(k)]
    c[k - 1] = p[0]
    for i in range(1, k):
        p_i = p[i]
        for j in range(k - 1 - (i - 1), k - 1):
            c[j] ^= gf_mul(p_i, c[j + 1])
        c[k - 1] ^= p_i
    for row in range(k):
        xx = p[row]
        t = 1
        b[k - 1] = 1
        for i in range(k - 1, 0, -1):
            b[i - 1] = c[i] ^ gf_mul(xx, b[i])
            t = gf_mul(xx, t) ^ b[i - 1]
        for col in range(k):
            src[col * k + row] = gf_mul(INVERSE[t], b[col])


def enc_matrix(k: int, m: int) -> list[list[int]]:
    """fec.c fec_new(k, n) with n = m."""
    tmp = [0] * (m * k)
    tmp[0] = 1
    for row in range(m - 1):
        for col in range(k):
            tmp[k + row * k + col] = GF_EXP[(row * col) % 255]
    top = tmp[: k * k]
    _invert_vdm(top, k)
    enc = [[0] * k for _ in range(m)]
    for r in range(k):
        enc[r][r] = 1
    for r in range(k, m):
        for c_ in range(k):
            acc = 0
            for t in range(k):
                acc ^= gf_mul(tmp[r * k + t], top[t * k + c_])
            enc[r][c_] = acc
    return enc


def _mul_table():
    import numpy as np
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(256):
        for b in range(256):
            t[a, b] = gf_mul(a, b)
    return t


_MT = None


def zfec_encode(data: bytes, k: int = 4, m: int = 8) -> tuple[bytes, int, int]:
    """encoding.rs:48-81 semantics (pad to 1024*k, contiguous shards)."""
    import numpy as np
    global _MT
    if _MT is None:
        _MT = _mul_table()
    unit = 1024 * k
    target = -(-len(data) // unit) * unit
    pad = target - len(data)
    C = target // k
    buf = np.zeros(target, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(data, dtype=np.uint8)
    shards = [buf[j * C:(j + 1) * C] for j in range(k)]
    E = enc_matrix(k, m)
    out = [s.copy() for s in shards]
    for i in range(k, m):
        acc = np.zeros(C, dtype=np.uint8)
        for j in range(k):
            acc ^= _MT[E[i][j]][shards[j]]
        out.append(acc)
    return b"".join(o.tobytes() for o in out), pad, C


# ---------------- BLAKE3 (CV-stack formulation) ----------------
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
MSG_PERMUTATION = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8
M32 = 0xFFFFFFFF


def _g(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = ((s[d] ^ s[a]) >> 16 | (s[d] ^ s[a]) << 16) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 12 | (s[b] ^ s[c]) << 20) & M32
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = ((s[d] ^ s[a]) >> 8 | (s[d] ^ s[a]) << 24) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 7 | (s[b] ^ s[c]) << 25) & M32


def compress(cv, block_words, counter, block_len, flags):
    s = list(cv) + IV[:4] + [counter & M32, (counter >> 32) & M32, block_len, flags]
    m = list(block_words)
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        if r < 6:
            m = [m[i] for i in MSG_PERMUTATION]
    return [s[i] ^ s[i + 8] for i in range(8)]


def _words(block: bytes) -> list[int]:
    block = block + b"\0" * (64 - len(block))
    return list(struct.unpack("<16I", block))


class _Output:
    def __init__(self, cv, words, counter, blen, flags):
        self.cv, self.words, self.counter, self.blen, self.flags = cv, words, counter, blen, flags

    def chaining_value(self):
        return compress(self.cv, self.words, self.counter, self.blen, self.flags)

    def root(self):
        return compress(self.cv, self.words, self.counter, self.blen, self.flags | ROOT)


def _chunk_output(chunk: bytes, counter: int) -> _Output:
    cv = IV[:]
    blocks = [chunk[i:i + 64] for i in range(0, len(chunk), 64)] or [b""]
    for bi, blk in enumerate(blocks):
        flags = (CHUNK_START if bi == 0 else 0) | (CHUNK_END if bi == len(blocks) - 1 else 0)
        if bi == len(blocks) - 1:
            return _Output(cv, _words(blk), counter, len(blk), flags)
        cv = compress(cv, _words(blk), counter, len(blk), flags)
    raise AssertionError


def _parent_output(l, r) -> _Output:
    return _Output(IV[:], l + r, 0, 64, PARENT)


def blake3(data: bytes) -> bytes:
    """Incremental hasher: push chunk CVs on a stack, merging completed subtrees."""
    stack = []
    chunks = [data[i:i + 1024] for i in range(0, len(data), 1024)] or [b""]
    total = 0
    for idx, ch in enumerate(chunks[:-1]):
        cv = _chunk_output(ch, idx).chaining_value()
        total = idx + 1
        t = total
        while t & 1 == 0:
            cv = _parent_output(stack.pop(), cv).chaining_value()
            t >>= 1
        stack.append(cv)
    out = _chunk_output(chunks[-1], len(chunks) - 1)
    while stack:
        out = _parent_output(stack.pop(), out.chaining_value())
    return struct.pack("<8I", *out.root())


# ---------------- bao combined encoding (explicit pre-order) ----------------
def bao_encode(data: bytes) -> tuple[bytes, bytes]:
    parts: list[bytes] = [struct.pack("<Q", len(data))]

    def rec(off: int, length: int, is_root: bool):
        if length <= 1024:
            o = _chunk_output(data[off:off + length], off // 1024)
            parts.append(data[off:off + length])
            return o.root() if is_root else o.chaining_value()
        full = (length - 1) // 1024
        left = 1024 * (1 << (full.bit_length() - 1))
        slot = len(parts)
        parts.append(b"")
        lcv = rec(off, left, False)
        rcv = rec(off + left, length - left, False)
        parts[slot] = struct.pack("<8I", *lcv) + struct.pack("<8I", *rcv)
        o = _parent_output(lcv, rcv)
        return o.root() if is_root else o.chaining_value()

    root = rec(0, len(data), True)
    return b"".join(parts), struct.pack("<8I", *root)


def bao_slice(encoded: bytes, start: int, length: int) -> bytes:
    """bao combined-encoding slice: header + pre-order parents/chunks whose
    subtree overlaps [start, start+length); at least one chunk; a start at or
    past the end selects the final chunk."""
    n = struct.unpack("<Q", encoded[:8])[0]
    chunks = max(1, -(-n // 1024))
    first = min(start // 1024, chunks - 1)
    last = max(first + 1, min(-(-(start + length) // 1024), chunks))  # exclusive
    out = [encoded[:8]]
    pos = 8

    def walk(c_lo, c_cnt):
        nonlocal pos
        if c_cnt == 1:
            size = min(1024, n - c_lo * 1024) if n else 0
            if first <= c_lo < last:
                out.append(encoded[pos:pos + size])
            pos += size
            return
        left = 1 << ((c_cnt - 1).bit_length() - 1)
        hit = c_lo < last and c_lo + c_cnt > first
        if hit:
            out.append(encoded[pos:pos + 64])
        pos += 64
        walk(c_lo, left)
        walk(c_lo + left, c_cnt - left)

    walk(0, chunks)
    return b"".join(out)
