"""The patched carbonado crate's device calls (carbonado-hip/reroute.patch
over carbonado-hip/src/lib.rs), replayed through ctypes.

This image has no cargo, so the Rust crate is never compiled here.  What the
`hip` feature executes is still fully determined by two texts: the patch
says which `carbonado_hip::` wrapper each reference function calls, and
lib.rs says which `chip_*` entry point (with which buffer sizes) each wrapper
calls.  This module makes exactly those C-ABI calls in that order, so the GPU
tests (tests/test_gpu_reroute.py) check the bytes a patched `carbonado`
returns, and tests/test_rust_shim.py checks (on CPU) that the call tables
below are the ones the two texts name.

The reference's host crates (snap 1.1, ecies 0.2) stay in Rust under the
patch; here the library's own host stages stand in for them
(chip_snap_compress / chip_ecies_encrypt with injected randomness), the
same bytes as the C oracle's restatement on incompressible input.
"""
from __future__ import annotations

import ctypes

from carbonado_amd import _lib
from carbonado_amd._lib import EciesInjectC, EncodeInfoC

FEC_K, FEC_M, SLICE_LEN, HASH_LEN = 4, 8, 1024, 32
ZFEC, BAO, ECIES, SNAPPY = 8, 4, 1, 2

# reference function -> the chip_* calls the patched crate makes for it, by
# the Format bits that are set (encoding.rs / decoding.rs under `hip`)
ENCODE_CALLS = {ZFEC | BAO: ["chip_encode"], ZFEC: ["chip_zfec_encode"], BAO: ["chip_bao_encode"], 0: []}
DECODE_CALLS = {ZFEC | BAO: ["chip_decode"], ZFEC: ["chip_zfec_decode"], BAO: ["chip_bao_decode"], 0: []}
SLICE_CALLS = {"scrub": ["chip_scrub"], "verify_slice": ["chip_bao_verify_slice"],
               "extract_slice": ["chip_bao_slice_len", "chip_bao_extract_slice"]}
# the `hip-stages` feature: every level in one chip_encode / chip_decode
STAGES_CALLS = ["chip_encode"], ["chip_decode"]
# round 5's patch (stage reroutes only): encode() at Zfec|Bao went zfec ->
# host Vec -> bao, decode() bao -> host Vec -> zfec
ENCODE_CALLS_R5 = {ZFEC | BAO: ["chip_zfec_encode", "chip_bao_encode"]}
DECODE_CALLS_R5 = {ZFEC | BAO: ["chip_bao_decode", "chip_zfec_decode"]}


class ChipStatus(Exception):
    def __init__(self, fn: str, rc: int):
        super().__init__(f"{fn}: status {rc}")
        self.fn, self.rc = fn, rc


def _L():
    return _lib.lib()


def _buf(n: int):
    return (ctypes.c_uint8 * max(n, 1))()


def _into_vec(fn: str, cap: int, call) -> bytes:
    """lib.rs into_vec: a fresh buffer of `cap`, the call, `len` bytes kept."""
    out = _buf(cap)
    ln = ctypes.c_uint64(0)
    rc = call(out, cap, ctypes.byref(ln))
    if rc != 0:
        raise ChipStatus(fn, rc)
    assert ln.value <= cap
    return bytes(out)[: ln.value]


# ---- the lib.rs wrappers the patch calls -------------------------------------

def zfec_encode(data: bytes) -> tuple[bytes, int, int]:
    total = _L().chip_zfec_encoded_len(len(data), FEC_K, FEC_M)
    out = _buf(total)
    pad, chunk = ctypes.c_uint32(), ctypes.c_uint32()
    rc = _L().chip_zfec_encode(FEC_K, FEC_M, data, len(data), out, total, ctypes.byref(pad), ctypes.byref(chunk))
    if rc:
        raise ChipStatus("chip_zfec_encode", rc)
    return bytes(out)[:total], pad.value, chunk.value


def zfec_decode(data: bytes, padding: int) -> bytes:
    cap = len(data) // FEC_M * FEC_K
    return _into_vec("chip_zfec_decode", cap, lambda o, c, l: _L().chip_zfec_decode(
        FEC_K, FEC_M, data, len(data), padding, o, c, l))


def bao_encode(data: bytes) -> tuple[bytes, bytes]:
    h = _buf(HASH_LEN)
    enc = _into_vec("chip_bao_encode", _L().chip_bao_encoded_len(len(data)),
                    lambda o, c, l: _L().chip_bao_encode(data, len(data), o, c, l, h))
    return enc, bytes(h)


def bao_decode(data: bytes, hash: bytes) -> bytes:
    return _into_vec("chip_bao_decode", len(data), lambda o, c, l: _L().chip_bao_decode(
        data, len(data), hash, len(hash), o, c, l))


def fused_encode(data: bytes, fmt: int = ZFEC | BAO) -> tuple[bytes, bytes, EncodeInfoC]:
    """carbonado_hip::encode(&[], &encrypted, 12, None)."""
    h = _buf(HASH_LEN)
    info = EncodeInfoC()
    enc = _into_vec("chip_encode", _L().chip_encode_max_len(len(data)), lambda o, c, l: _L().chip_encode(
        fmt, b"", 0, None, data, len(data), o, c, l, h, ctypes.byref(info)))
    return enc, bytes(h), info


def fused_decode(hash: bytes, data: bytes, padding: int, fmt: int = ZFEC | BAO) -> bytes:
    """carbonado_hip::decode(&[], hash, input, padding, 12) (into_vec_grow)."""
    def call(cap):
        return _into_vec("chip_decode", cap, lambda o, c, l: _L().chip_decode(
            b"", 0, hash, len(hash), data, len(data), padding, fmt, o, c, l))
    return call(max(len(data), 1024))


def scrub(data: bytes, hash: bytes, padding: int, chunk_len: int) -> bytes:
    return _into_vec("chip_scrub", len(data), lambda o, c, l: _L().chip_scrub(
        data, len(data), hash, len(hash), padding, chunk_len, o, c, l))


def verify_slice(hash: bytes, data: bytes, index: int, count: int) -> bytes:
    cap = min(count * SLICE_LEN, len(data))
    return _into_vec("chip_bao_verify_slice", cap, lambda o, c, l: _L().chip_bao_verify_slice(
        hash, len(hash), data, len(data), index, count, o, c, l))


def extract_slice(encoded: bytes, index: int) -> bytes:
    content = int.from_bytes(encoded[:8], "little")
    cap = _L().chip_bao_slice_len(content, index * SLICE_LEN, SLICE_LEN)
    return _into_vec("chip_bao_extract_slice", cap, lambda o, c, l: _L().chip_bao_extract_slice(
        encoded, len(encoded), index, SLICE_LEN, o, c, l))


# ---- the host crates (Rust under the patch; the library's stages stand in) ---

def host_encode(data: bytes, fmt: int, pubkey: bytes, eph_sk: bytes, nonce: bytes) -> tuple[bytes, int, int]:
    cur, bc, be = data, 0, 0
    if fmt & SNAPPY:
        cur = _into_vec("chip_snap_compress", _L().chip_snap_max_len(len(cur)), lambda o, c, l: _L().chip_snap_compress(
            cur, len(cur), o, c, l))
        bc = len(cur)
    if fmt & ECIES:
        e, nn = (ctypes.c_uint8 * 32).from_buffer_copy(eph_sk), (ctypes.c_uint8 * 16).from_buffer_copy(nonce)
        inj = EciesInjectC(ctypes.addressof(e), ctypes.addressof(nn))
        src = cur
        cur = _into_vec("chip_ecies_encrypt", len(src) + 97, lambda o, c, l: _L().chip_ecies_encrypt(
            pubkey, len(pubkey), ctypes.byref(inj), src, len(src), o, c, l))
        be = len(cur)
    return cur, bc, be


def host_decode(data: bytes, fmt: int, secret_key: bytes) -> bytes:
    cur = data
    if fmt & ECIES:
        src = cur
        cur = _into_vec("chip_ecies_decrypt", len(src), lambda o, c, l: _L().chip_ecies_decrypt(
            secret_key, len(secret_key), src, len(src), o, c, l))
    if fmt & SNAPPY:
        src = cur
        cap = max(1024, 2 * len(src))
        try:
            cur = _into_vec("chip_snap_decompress", cap, lambda o, c, l: _L().chip_snap_decompress(
                src, len(src), o, c, l))
        except ChipStatus:
            cur = _into_vec("chip_snap_decompress", 64 * len(src) + 1024, lambda o, c, l: _L().chip_snap_decompress(
                src, len(src), o, c, l))
    return cur


# ---- the patched glue (encoding.rs:86-172, decoding.rs:80-114) ---------------

def encode(data: bytes, level: int, pubkey: bytes = b"", eph_sk: bytes = bytes(32), nonce: bytes = bytes(16),
           r5: bool = False) -> tuple[bytes, bytes, dict, list]:
    """(stream, hash, EncodeInfo fields, chip_* calls made).  r5: round 5's
    patch (zfec then bao at Zfec|Bao: two device round trips)."""
    cur, bc, be = host_encode(data, level, pubkey, eph_sk, nonce)
    calls = []
    zb = level & (ZFEC | BAO)
    if zb == ZFEC | BAO and not r5:
        enc, h, zi = fused_encode(cur)
        calls.append("chip_encode")
        info = dict(padding_len=zi.padding_len, chunk_len=zi.chunk_len, bytes_ecc=zi.bytes_ecc,
                    bytes_verifiable=zi.bytes_verifiable, verifiable_slice_count=zi.verifiable_slice_count,
                    chunk_slice_count=zi.chunk_slice_count)
    else:
        pad = chunk = ecc = vsc = csc = bv = 0
        if zb & ZFEC:
            cur, pad, chunk = zfec_encode(cur)
            calls.append("chip_zfec_encode")
            ecc = len(cur)
            vsc = (ecc // SLICE_LEN) & 0xFFFF
            csc = vsc // 8
        h = bytes(32)
        if zb & BAO:
            cur, h = bao_encode(cur)
            calls.append("chip_bao_encode")
            bv = len(cur)
        enc = cur
        info = dict(padding_len=pad, chunk_len=chunk, bytes_ecc=ecc, bytes_verifiable=bv,
                    verifiable_slice_count=vsc, chunk_slice_count=csc)
    info.update(input_len=len(data), output_len=len(enc), bytes_compressed=bc, bytes_encrypted=be)
    return enc, h, info, calls


def decode(secret_key: bytes, hash: bytes, data: bytes, padding: int, level: int,
           r5: bool = False) -> tuple[bytes, list]:
    calls = []
    zb = level & (ZFEC | BAO)
    if zb == ZFEC | BAO and not r5:
        cur = fused_decode(hash, data, padding)
        calls.append("chip_decode")
    else:
        cur = data
        if zb & BAO:
            cur = bao_decode(cur, hash)
            calls.append("chip_bao_decode")
        if zb & ZFEC:
            cur = zfec_decode(cur, padding)
            calls.append("chip_zfec_decode")
    return host_decode(cur, level, secret_key), calls


# ---- the `hip-stages` feature: encode()/decode() whole in the library --------

def encode_stages(data: bytes, level: int, pubkey: bytes = b"", eph_sk: bytes = bytes(32),
                  nonce: bytes = bytes(16)) -> tuple[bytes, bytes, EncodeInfoC]:
    """carbonado_hip::encode(pubkey, input, format, None) (inject given here
    for bit-exact checks)."""
    h = _buf(HASH_LEN)
    info = EncodeInfoC()
    e, nn = (ctypes.c_uint8 * 32).from_buffer_copy(eph_sk), (ctypes.c_uint8 * 16).from_buffer_copy(nonce)
    inj = EciesInjectC(ctypes.addressof(e), ctypes.addressof(nn))
    cap = _L().chip_encode_max_len(_L().chip_snap_max_len(len(data)) + 97)
    enc = _into_vec("chip_encode", cap, lambda o, c, l: _L().chip_encode(
        level, pubkey, len(pubkey), ctypes.byref(inj), data, len(data), o, c, l, h, ctypes.byref(info)))
    return enc, bytes(h), info


def decode_stages(secret_key: bytes, hash: bytes, data: bytes, padding: int, level: int, n_hint: int) -> bytes:
    """carbonado_hip::decode(secret_key, hash, input, padding, format)."""
    return _into_vec("chip_decode", max(len(data), 1024, n_hint + 1024), lambda o, c, l: _L().chip_decode(
        secret_key, len(secret_key), hash, len(hash), data, len(data), padding, level, o, c, l))
