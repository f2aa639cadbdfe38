"""encoding (mirror of /root/reference/src/encoding.rs) through
libcarbonado_hip: zfec and bao on the MI355X, snap and ecies as the
library's host stages (host_stages.cpp)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._buf import OutBytes, as_u8, check, ptr
from .constants import FEC_K, FEC_M, Format
from .structs import EncodeInfo, Encoded


def _inject(ephemeral_sk: bytes | None, nonce: bytes | None):
    """chip_ecies_inject for test determinism; None = the reference's RNG."""
    if ephemeral_sk is None and nonce is None:
        return None, ()
    keep = tuple(as_u8(x) for x in (ephemeral_sk, nonce) if x is not None)
    inj = _lib.EciesInjectC(
        ptr(as_u8(ephemeral_sk)) if ephemeral_sk is not None else None,
        ptr(as_u8(nonce)) if nonce is not None else None)
    if ephemeral_sk is not None:
        assert len(ephemeral_sk) == 32
    if nonce is not None:
        assert len(nonce) == 16
    return inj, keep


def snap(input) -> bytes:
    """encoding.rs:16-28: snap::write::FrameEncoder output."""
    a = as_u8(input)
    L = _lib.lib()
    cap = L.chip_snap_max_len(a.size)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    olen = ctypes.c_uint64()
    check(L.chip_snap_compress(ptr(a), a.size, ptr(out), cap, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def ecies(pubkey: bytes, input, *, ephemeral_sk: bytes | None = None, nonce: bytes | None = None) -> bytes:
    """encoding.rs:30-36: ecies::encrypt(pubkey, input); n + 97 bytes.
    `ephemeral_sk`/`nonce` inject the two random values (tests only)."""
    a = as_u8(input)
    pk = as_u8(pubkey)
    cap = a.size + 97
    out = np.empty(cap, dtype=np.uint8)
    olen = ctypes.c_uint64()
    inj, _keep = _inject(ephemeral_sk, nonce)
    check(_lib.lib().chip_ecies_encrypt(ptr(pk), pk.size, ctypes.byref(inj) if inj is not None else None,
                                        ptr(a), a.size, ptr(out), cap, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def public_key(secret_key: bytes) -> bytes:
    """secp256k1 public key (65 bytes, uncompressed) of a 32-byte secret."""
    sk = as_u8(secret_key)
    out = np.empty(65, dtype=np.uint8)
    check(_lib.lib().chip_ecies_public_key(ptr(sk), ptr(out)))
    return out.tobytes()


def zfec(input, k: int = FEC_K, m: int = FEC_M) -> tuple[bytes, int, int]:
    """encoding.rs:46-81 → (encoded shard-major bytes, padding_len, chunk_len)."""
    a = as_u8(input)
    L = _lib.lib()
    total = L.chip_zfec_encoded_len(a.size, k, m)
    out = OutBytes(total)
    pad, chunk = ctypes.c_uint32(), ctypes.c_uint32()
    check(L.chip_zfec_encode(k, m, ptr(a), a.size, out.ptr(), total, ctypes.byref(pad), ctypes.byref(chunk)))
    return out.result(total), pad.value, chunk.value


def bao(input) -> tuple[bytes, bytes]:
    """encoding.rs:38-44 → (bao combined encoding, 32-byte root hash)."""
    a = as_u8(input)
    L = _lib.lib()
    total = L.chip_bao_encoded_len(a.size)
    out = OutBytes(total)
    h = np.empty(32, dtype=np.uint8)
    olen = ctypes.c_uint64()
    check(L.chip_bao_encode(ptr(a), a.size, out.ptr(), total, ctypes.byref(olen), ptr(h)))
    return out.result(olen.value), h.tobytes()


def blake3(input) -> bytes:
    """BLAKE3 hash (== the bao root hash) computed on the device."""
    a = as_u8(input)
    h = np.empty(32, dtype=np.uint8)
    check(_lib.lib().chip_blake3(ptr(a), a.size, ptr(h)))
    return h.tobytes()


def encode(pubkey: bytes, input, format: int, *, ephemeral_sk: bytes | None = None,
           nonce: bytes | None = None) -> Encoded:
    """encoding.rs:86-172 `encode(pubkey, input, format) -> Encoded`.

    snap → ecies run as host stages, then zfec → bao device-resident (the
    zfec output never returns to the host).  `pubkey` is used by the ECIES
    stage only; `ephemeral_sk`/`nonce` inject its random values (tests)."""
    a = as_u8(input)
    pk = as_u8(pubkey)
    L = _lib.lib()
    fmt = int(Format(format))
    if fmt & Format.Snappy:
        cap = L.chip_encode_max_len(a.size)  # compressed size known only afterwards
    else:  # exact: the output becomes the returned bytes without a copy
        cap = a.size + 97 if fmt & Format.Ecies else a.size
        if fmt & Format.Zfec:
            cap = L.chip_zfec_encoded_len(cap, FEC_K, FEC_M)
        if fmt & Format.Bao:
            cap = L.chip_bao_encoded_len(cap)
    out = OutBytes(cap)
    h = np.empty(32, dtype=np.uint8)
    olen = ctypes.c_uint64()
    info = _lib.EncodeInfoC()
    inj, _keep = _inject(ephemeral_sk, nonce)
    check(L.chip_encode(fmt, ptr(pk) if pk.size else None, pk.size,
                        ctypes.byref(inj) if inj is not None else None, ptr(a), a.size, out.ptr(), cap,
                        ctypes.byref(olen), ptr(h), ctypes.byref(info)))
    return Encoded(out.result(olen.value), h.tobytes(), EncodeInfo.from_c(info))
