"""utils (mirror of the hot-path helpers in /root/reference/src/utils.rs)."""
from __future__ import annotations

import ctypes

from . import _lib
from .constants import FEC_K, HASH_SIZE
from .error import HashDecodeError


def calc_padding_len(input_len: int, k: int = FEC_K) -> tuple[int, int]:
    """utils.rs:47-58 → (padding_len, chunk_size).  The reference computes this
    in f64; the C-ABI uses exact integer maths (identical for every length)."""
    pad = ctypes.c_uint32()
    chunk = ctypes.c_uint32()
    rc = _lib.lib().chip_calc_padding_len(input_len, k, ctypes.byref(pad), ctypes.byref(chunk))
    if rc:
        raise ValueError("k must be >= 1")
    return pad.value, chunk.value


def decode_bao_hash(hash: bytes) -> bytes:
    """utils.rs:37-45: exactly 32 bytes, else HashDecodeError(32, len)."""
    if len(hash) != HASH_SIZE:
        raise HashDecodeError(HASH_SIZE, len(hash))
    return bytes(hash)


def encode_bao_hash(hash: bytes) -> str:
    """utils.rs:31-35: lowercase hex."""
    return bytes(hash).hex()
