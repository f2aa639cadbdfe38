"""encoding (mirror of /root/reference/src/encoding.rs), hot-path stages on
the MI355X through libcarbonado_hip.  Snappy/ECIES are host stages outside
this path: their format bits raise UnsupportedFormat."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._buf import as_u8, check, ptr
from .constants import FEC_K, FEC_M, Format
from .structs import EncodeInfo, Encoded


def zfec(input, k: int = FEC_K, m: int = FEC_M) -> tuple[bytes, int, int]:
    """encoding.rs:46-81 → (encoded shard-major bytes, padding_len, chunk_len)."""
    a = as_u8(input)
    L = _lib.lib()
    total = L.chip_zfec_encoded_len(a.size, k, m)
    out = np.empty(max(total, 1), dtype=np.uint8)
    pad, chunk = ctypes.c_uint32(), ctypes.c_uint32()
    check(L.chip_zfec_encode(k, m, ptr(a), a.size, ptr(out), total, ctypes.byref(pad), ctypes.byref(chunk)))
    return out[:total].tobytes(), pad.value, chunk.value


def bao(input) -> tuple[bytes, bytes]:
    """encoding.rs:38-44 → (bao combined encoding, 32-byte root hash)."""
    a = as_u8(input)
    L = _lib.lib()
    total = L.chip_bao_encoded_len(a.size)
    out = np.empty(total, dtype=np.uint8)
    h = np.empty(32, dtype=np.uint8)
    olen = ctypes.c_uint64()
    check(L.chip_bao_encode(ptr(a), a.size, ptr(out), total, ctypes.byref(olen), ptr(h)))
    return out[: olen.value].tobytes(), h.tobytes()


def blake3(input) -> bytes:
    """BLAKE3 hash (== the bao root hash) computed on the device."""
    a = as_u8(input)
    h = np.empty(32, dtype=np.uint8)
    check(_lib.lib().chip_blake3(ptr(a), a.size, ptr(h)))
    return h.tobytes()


def encode(pubkey: bytes, input, format: int) -> Encoded:
    """encoding.rs:86-172 `encode(pubkey, input, format) -> Encoded`.

    The zfec → bao chain runs device-resident (the zfec output never returns
    to the host).  `pubkey` is only used by the ECIES stage (out of scope)."""
    del pubkey
    a = as_u8(input)
    L = _lib.lib()
    cap = L.chip_encode_max_len(a.size)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    h = np.empty(32, dtype=np.uint8)
    olen = ctypes.c_uint64()
    info = _lib.EncodeInfoC()
    check(L.chip_encode(int(Format(format)), ptr(a), a.size, ptr(out), cap, ctypes.byref(olen), ptr(h),
                        ctypes.byref(info)))
    return Encoded(out[: olen.value].tobytes(), h.tobytes(), EncodeInfo.from_c(info))
