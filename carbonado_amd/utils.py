"""utils (mirror of the hot-path helpers in /root/reference/src/utils.rs)."""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from ._buf import OutBytes, as_u8, check, ptr
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


class BaoHash(bytes):
    """utils.rs:72-102 `BaoHash(bao::Hash)`: 32 bytes, Display = lowercase hex."""

    def __new__(cls, value):
        b = bytes(value)[:32]
        if len(b) != HASH_SIZE:
            raise HashDecodeError(HASH_SIZE, len(b))
        return super().__new__(cls, b)

    def to_bytes(self) -> bytes:
        return bytes(self)

    def __str__(self) -> str:
        return self.hex()


class BaoHasher:
    """utils.rs:104-137 `BaoHasher`: a thread-safe append-only bao hasher.

    update() appends to an HBM buffer on the device; finalize() runs the bao
    kernels over everything appended (root hash == BLAKE3 of the content);
    read_all() returns the combined encoding.  Locking is inside the library
    (one mutex per hasher, as the reference's RwLock)."""

    def __init__(self):
        h = ctypes.c_void_p()
        check(_lib.lib().chip_bao_hasher_new(ctypes.byref(h)))
        self._h = h
        self._free_lock = threading.Lock()

    @classmethod
    def new(cls) -> "BaoHasher":
        """utils.rs:110-120 `BaoHasher::new() -> Arc<Self>` (Python objects are shared by reference)."""
        return cls()

    def update(self, buf) -> None:
        a = as_u8(buf)
        check(_lib.lib().chip_bao_hasher_update(self._h, ptr(a), a.size))

    def finalize(self) -> BaoHash:
        out = np.empty(32, np.uint8)
        check(_lib.lib().chip_bao_hasher_finalize(self._h, ptr(out)))
        return BaoHash(out.tobytes())

    def __len__(self) -> int:
        return int(_lib.lib().chip_bao_hasher_len(self._h))

    def read_all(self) -> bytes:
        L = _lib.lib()
        need = ctypes.c_uint64()
        L.chip_bao_hasher_read_all(self._h, None, 0, ctypes.byref(need))  # size query
        out = OutBytes(need.value)
        olen = ctypes.c_uint64()
        check(L.chip_bao_hasher_read_all(self._h, out.ptr(), need.value, ctypes.byref(olen)))
        return out.result(olen.value)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                with self._free_lock:
                    _lib.lib().chip_bao_hasher_free(h)
                    self._h = ctypes.c_void_p()
            except Exception:  # interpreter shutdown: the library may already be gone
                pass
