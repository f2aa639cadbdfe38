"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU oracle restates the reference path (see carbonado_oracle.h for
file:line citations).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, as the checker; the product never does.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        if not LIB.exists():
            build()
        l = ctypes.CDLL(str(LIB))
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        l.orc_blake3.argtypes = [vp, u64, vp]
        l.orc_fec_enc_matrix.argtypes = [ctypes.c_uint, ctypes.c_uint, vp]
        l.orc_zfec_encode.argtypes = [ctypes.c_uint, ctypes.c_uint, vp, u64, vp, u64,
                                      ctypes.POINTER(u32), ctypes.POINTER(u32)]
        l.orc_zfec_decode_shares.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(vp),
                                             ctypes.POINTER(u32), ctypes.c_uint, u64, u32, vp, u64,
                                             ctypes.POINTER(u64)]
        l.orc_zfec_decode.argtypes = [ctypes.c_uint, ctypes.c_uint, vp, u64, u32, vp, u64, ctypes.POINTER(u64)]
        l.orc_bao_encoded_len.argtypes = [u64]
        l.orc_bao_encoded_len.restype = u64
        l.orc_bao_encode.argtypes = [vp, u64, vp, u64, vp]
        l.orc_bao_decode.argtypes = [vp, u64, vp, u64, vp, u64, ctypes.POINTER(u64)]
        l.orc_encode_max_len.argtypes = [u64]
        l.orc_encode_max_len.restype = u64
        l.orc_encode.argtypes = [ctypes.c_uint8, vp, u64, vp, u64, ctypes.POINTER(u64), vp, vp]
        l.orc_decode.argtypes = [vp, u64, vp, u64, u32, ctypes.c_uint8, vp, u64, ctypes.POINTER(u64)]
        l.orc_fill_object.argtypes = [u64, u64, vp, u64]
        l.orc_calc_padding_len.argtypes = [u64, ctypes.c_uint, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        l.orc_crc32c.argtypes = [vp, u64]
        l.orc_crc32c.restype = u32
        l.orc_snap_max_len.argtypes = [u64]
        l.orc_snap_max_len.restype = u64
        l.orc_snap_compress.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64)]
        l.orc_snap_decompress.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64)]
        l.orc_sha256.argtypes = [vp, u64, vp]
        l.orc_hmac_sha256.argtypes = [vp, u64, vp, u64, vp]
        l.orc_ecies_public_key.argtypes = [vp, vp]
        l.orc_ecies_encrypt.argtypes = [vp, u64, vp, vp, vp, u64, vp, u64, ctypes.POINTER(u64)]
        l.orc_ecies_decrypt.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64)]
        l.orc_encode_full.argtypes = [ctypes.c_uint8, vp, u64, vp, vp, vp, u64, vp, u64, ctypes.POINTER(u64), vp, vp]
        _L = l
    return _L


def _u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data if a.size else 0)


class OracleError(Exception):
    def __init__(self, status: int):
        super().__init__(f"oracle status {status}")
        self.status = status


def _chk(rc: int) -> None:
    if rc:
        raise OracleError(rc)


def blake3(data) -> bytes:
    a = _u8(data)
    out = np.empty(32, np.uint8)
    lib().orc_blake3(_p(a), a.size, _p(out))
    return out.tobytes()


def enc_matrix(k: int, m: int) -> np.ndarray:
    out = np.empty(k * m, np.uint8)
    _chk(lib().orc_fec_enc_matrix(k, m, _p(out)))
    return out.reshape(m, k)


def calc_padding_len(n: int, k: int = 4) -> tuple[int, int]:
    p, c = ctypes.c_uint32(), ctypes.c_uint32()
    lib().orc_calc_padding_len(n, k, ctypes.byref(p), ctypes.byref(c))
    return p.value, c.value


def zfec_encode(data, k: int = 4, m: int = 8) -> tuple[bytes, int, int]:
    a = _u8(data)
    pad, C = calc_padding_len(a.size, k)
    out = np.empty(max(m * C, 1), np.uint8)
    p, c = ctypes.c_uint32(), ctypes.c_uint32()
    _chk(lib().orc_zfec_encode(k, m, _p(a), a.size, _p(out), m * C, ctypes.byref(p), ctypes.byref(c)))
    return out[: m * C].tobytes(), p.value, c.value


def zfec_decode_shares(shares, idx, padding: int, k: int = 4, m: int = 8) -> bytes:
    arrs = [_u8(s) for s in shares]
    C = arrs[0].size
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    cidx = (ctypes.c_uint32 * n)(*idx)
    out = np.empty(max(k * C, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_zfec_decode_shares(k, m, ptrs, cidx, n, C, padding, _p(out), k * C, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def zfec_decode(data, padding: int, k: int = 4, m: int = 8) -> bytes:
    a = _u8(data)
    out = np.empty(max(a.size, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_zfec_decode(k, m, _p(a), a.size, padding, _p(out), a.size, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def bao_encode(data) -> tuple[bytes, bytes]:
    a = _u8(data)
    n = lib().orc_bao_encoded_len(a.size)
    out = np.empty(n, np.uint8)
    h = np.empty(32, np.uint8)
    _chk(lib().orc_bao_encode(_p(a), a.size, _p(out), n, _p(h)))
    return out.tobytes(), h.tobytes()


def bao_decode(enc, hash: bytes) -> bytes:
    a = _u8(enc)
    h = _u8(hash)
    out = np.empty(max(a.size, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_bao_decode(_p(a), a.size, _p(h), h.size, _p(out), a.size, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


class EncodeInfoC(ctypes.Structure):
    _fields_ = [("input_len", ctypes.c_uint32), ("output_len", ctypes.c_uint32),
                ("bytes_compressed", ctypes.c_uint32), ("compression_factor", ctypes.c_float),
                ("bytes_encrypted", ctypes.c_uint32), ("bytes_ecc", ctypes.c_uint32),
                ("bytes_verifiable", ctypes.c_uint32), ("amplification_factor", ctypes.c_float),
                ("padding_len", ctypes.c_uint32), ("chunk_len", ctypes.c_uint32),
                ("verifiable_slice_count", ctypes.c_uint16), ("chunk_slice_count", ctypes.c_uint16)]


def encode(data, fmt: int) -> tuple[bytes, bytes, dict]:
    a = _u8(data)
    cap = lib().orc_encode_max_len(a.size)
    out = np.empty(max(cap, 1), np.uint8)
    h = np.empty(32, np.uint8)
    olen = ctypes.c_uint64()
    info = EncodeInfoC()
    _chk(lib().orc_encode(fmt, _p(a), a.size, _p(out), cap, ctypes.byref(olen), _p(h), ctypes.byref(info)))
    return out[: olen.value].tobytes(), h.tobytes(), {f: getattr(info, f) for f, _ in info._fields_}


def decode(hash: bytes, data, padding: int, fmt: int) -> bytes:
    a = _u8(data)
    h = _u8(hash)
    out = np.empty(max(a.size, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_decode(_p(h), h.size, _p(a), a.size, padding, fmt, _p(out), a.size, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def fill_object(seed: int, obj: int, n: int) -> np.ndarray:
    out = np.empty(n, np.uint8)
    lib().orc_fill_object(seed, obj, _p(out), n)
    return out


def encode_full(data, fmt: int, pubkey: bytes | None = None, eph_sk: bytes | None = None,
                nonce: bytes | None = None) -> tuple[bytes, bytes, dict]:
    """encoding.rs:86-172 with every format bit: the host stages restated in
    host_oracle (snap, ecies with injected randomness), then this module's C
    restatement of zfec -> bao.  EncodeInfo factors in f32 as encoding.rs:149-151."""
    from . import host_oracle as H
    data = bytes(_u8(data))
    cur, bc, be = H.host_encode(data, fmt, pubkey, eph_sk, nonce)
    enc, h, info = encode(cur, fmt & 12)
    n = np.float32(len(data))
    with np.errstate(divide="ignore", invalid="ignore"):
        info["compression_factor"] = float(np.float32(bc) / n)
        info["amplification_factor"] = float(np.float32(info["bytes_verifiable"]) / n)
    info.update(input_len=len(data), bytes_compressed=bc, bytes_encrypted=be)
    return enc, h, info


def decode_full(secret: bytes | None, hash: bytes, data, padding: int, fmt: int) -> bytes:
    """decoding.rs:80-114: bao -> zfec (C restatement), then ecies -> snap."""
    from . import host_oracle as H
    cur = decode(hash, data, padding, fmt & 12) if fmt & 12 else bytes(_u8(data))
    return H.host_decode(cur, fmt, secret)


# ---- C restatement of the host stages (host_oracle.c): full-size checker ----
def c_snap_compress(data) -> bytes:
    a = _u8(data)
    cap = lib().orc_snap_max_len(a.size) + 1
    out = np.empty(cap, np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_snap_compress(_p(a), a.size, _p(out), cap, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def c_snap_decompress(data, cap: int) -> bytes:
    a = _u8(data)
    out = np.empty(max(cap, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_snap_decompress(_p(a), a.size, _p(out), cap, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def c_ecies_encrypt(pub: bytes, data, eph_sk: bytes, nonce: bytes) -> bytes:
    a, pk = _u8(data), _u8(pub)
    e, nn = _u8(eph_sk), _u8(nonce)
    out = np.empty(a.size + 97, np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_ecies_encrypt(_p(pk), pk.size, _p(e), _p(nn), _p(a), a.size, _p(out), out.size, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def c_ecies_decrypt(sk: bytes, data) -> bytes:
    a, k = _u8(data), _u8(sk)
    out = np.empty(max(a.size - 97, 1), np.uint8)
    olen = ctypes.c_uint64()
    _chk(lib().orc_ecies_decrypt(_p(k), _p(a), a.size, _p(out), out.size, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def c_public_key(sk: bytes) -> bytes:
    k = _u8(sk)
    out = np.empty(65, np.uint8)
    _chk(lib().orc_ecies_public_key(_p(k), _p(out)))
    return out.tobytes()


def c_encode_full(data, fmt: int, pubkey: bytes = b"", eph_sk: bytes = bytes(32), nonce: bytes = bytes(16)):
    """encoding.rs:86-172 for every format bit, all in C (snap, ecies with the
    injected ephemeral key and nonce, zfec, bao)."""
    a, pk = _u8(data), _u8(pubkey)
    e, nn = _u8(eph_sk), _u8(nonce)
    cap = lib().orc_encode_max_len(lib().orc_snap_max_len(a.size) + 97 + a.size) + 1
    out = np.empty(cap, np.uint8)
    h = np.empty(32, np.uint8)
    olen = ctypes.c_uint64()
    info = EncodeInfoC()
    _chk(lib().orc_encode_full(fmt, _p(pk), pk.size, _p(e), _p(nn), _p(a), a.size, _p(out), cap, ctypes.byref(olen),
                               _p(h), ctypes.byref(info)))
    return out[: olen.value].tobytes(), h.tobytes(), {f: getattr(info, f) for f, _ in info._fields_}
