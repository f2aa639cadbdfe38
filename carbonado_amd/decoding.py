"""decoding (mirror of /root/reference/src/decoding.rs), hot-path stages on
the MI355X through libcarbonado_hip."""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib
from ._buf import OutBytes, as_u8, check, ptr
from .constants import FEC_K, FEC_M, HASH_SIZE, Format
from .error import HashDecodeError


def zfec_chunks(chunks: Sequence, padding: int, indices: Sequence[int] | None = None,
                k: int = FEC_K, m: int = FEC_M) -> bytes:
    """decoding.rs:21-32.  With `indices=None` the shares are numbered by
    position exactly as the reference does (decoding.rs:24-25); pass the true
    share indices to decode after losing data shards."""
    arrs = [as_u8(c) for c in chunks]
    if not arrs:
        from .error import ZfecError
        raise ZfecError("no chunks")
    C = arrs[0].size
    if any(x.size != C for x in arrs):
        from .error import ZfecError
        raise ZfecError("chunks differ in length")
    idx = list(range(len(arrs))) if indices is None else list(indices)
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[x.ctypes.data if x.size else 0 for x in arrs])
    cidx = (ctypes.c_uint32 * n)(*idx)
    olen_max = k * C
    out = OutBytes(olen_max - padding if 0 <= padding <= olen_max else olen_max)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_zfec_decode_shares(k, m, ptrs, cidx, n, C, padding, out.ptr(), out.cap,
                                             ctypes.byref(olen)))
    return out.result(olen.value)


def zfec(input, padding: int, k: int = FEC_K, m: int = FEC_M) -> bytes:
    """decoding.rs:34-51: m contiguous shards (len % m == 0 else UnevenZfecChunks)."""
    a = as_u8(input)
    cap = (a.size // m) * k if m else 0
    out = OutBytes(cap - padding if 0 <= padding <= cap else cap)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_zfec_decode(k, m, ptr(a), a.size, padding, out.ptr(), out.cap, ctypes.byref(olen)))
    return out.result(olen.value)


def bao(input, hash: bytes) -> bytes:
    """decoding.rs:53-60: verify the whole stream against `hash`, return content."""
    if len(hash) != HASH_SIZE:
        raise HashDecodeError(HASH_SIZE, len(hash))
    a = as_u8(input)
    n = int.from_bytes(a[:8].tobytes(), "little") if a.size >= 8 else 0
    cap = min(n, a.size)
    out = OutBytes(cap)
    h = as_u8(hash)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_bao_decode(ptr(a), a.size, ptr(h), h.size, out.ptr(), cap, ctypes.byref(olen)))
    return out.result(olen.value)


def ecies(input, secret_key: bytes) -> bytes:
    """decoding.rs:62-68: ecies::decrypt(secret_key, input)."""
    a = as_u8(input)
    sk = as_u8(secret_key)
    cap = max(a.size - 97, 0)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_ecies_decrypt(ptr(sk), sk.size, ptr(a), a.size, ptr(out), cap, ctypes.byref(olen)))
    return out[: olen.value].tobytes()


def decoded_cap(a: np.ndarray, padding: int, fmt: Format) -> int:
    """Output buffer for decode(): the exact size unless Snappy is on (its
    size is known only after parsing: a first guess, grown on demand)."""
    if fmt & Format.Snappy:
        return a.size * 3 + 1024
    cap = a.size
    if fmt & Format.Bao:
        cap = min(int.from_bytes(a[:8].tobytes(), "little"), a.size) if a.size >= 8 else 0
    if fmt & Format.Zfec:
        cap = max((cap // FEC_M) * FEC_K - padding, 0)
    if fmt & Format.Ecies:
        cap = max(cap - 97, 0)
    return cap


def _grow_call(fn, cap: int) -> bytes:
    """Call fn(out, cap, olen); on BUFFER_TOO_SMALL retry once with the size
    the library reports (snappy output size is known only after parsing)."""
    from .error import BufferTooSmall
    for _ in range(2):
        out = OutBytes(cap)
        olen = ctypes.c_uint64()
        st = fn(out.ptr(), cap, olen)
        if st == BufferTooSmall.status and olen.value > cap:
            cap = olen.value
            continue
        check(st)
        return out.result(olen.value)
    check(st)


def snap(input) -> bytes:
    """decoding.rs:70-77: snap::read::FrameDecoder::read_to_end."""
    a = as_u8(input)
    return _grow_call(lambda out, cap, olen: _lib.lib().chip_snap_decompress(ptr(a), a.size, out, cap,
                                                                             ctypes.byref(olen)),
                      2 * a.size + 1024)


def decode(secret_key: bytes, hash: bytes, input, padding: int, format: int) -> bytes:
    """decoding.rs:80-114 `decode(secret_key, hash, input, padding, format)`:
    bao → zfec on the device, then ecies → snap as host stages."""
    a = as_u8(input)
    h = as_u8(hash)
    sk = as_u8(secret_key)
    fmt = Format(format)
    cap = decoded_cap(a, padding, fmt)
    return _grow_call(lambda out, c, olen: _lib.lib().chip_decode(
        ptr(sk) if sk.size else None, sk.size, ptr(h), h.size, ptr(a), a.size, padding, int(fmt), out, c,
        ctypes.byref(olen)), cap)


def extract_slice(encoded, index: int, slice_len: int = 1024) -> bytes:
    """decoding.rs:116-127 `extract_slice(encoded, index)`: the bao slice
    (header, parents on the path, chunks) of 1 KiB slice `index`.  The
    reference multiplies `index * SLICE_LEN` in u16 (wraps for index >= 64);
    this takes the index as an unbounded integer."""
    a = as_u8(encoded)
    n = int.from_bytes(a[:8].tobytes(), "little") if a.size >= 8 else 0
    L = _lib.lib()
    cap = L.chip_bao_slice_len(n, index * 1024, slice_len) if a.size >= 8 else 0
    out = OutBytes(cap)
    olen = ctypes.c_uint64()
    check(L.chip_bao_extract_slice(ptr(a), a.size, index, slice_len, out.ptr(), cap, ctypes.byref(olen)))
    return out.result(olen.value)


def verify_slice(hash: bytes, input, index: int, count: int) -> bytes:
    """decoding.rs:129-149 `verify_slice(hash, input, index, count)`: verify
    `count` 1 KiB slices from slice `index` of the combined encoding and return
    their content (the nodes are re-hashed on the device)."""
    if len(hash) != HASH_SIZE:
        raise HashDecodeError(HASH_SIZE, len(hash))
    a = as_u8(input)
    h = as_u8(hash)
    cap = count * 1024
    out = OutBytes(cap)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_bao_verify_slice(ptr(h), h.size, ptr(a), a.size, index, count, out.ptr(), cap,
                                           ctypes.byref(olen)))
    return out.result(olen.value)


def scrub(input, hash: bytes, encode_info) -> bytes:
    """decoding.rs:151-212 `scrub(input, hash, encode_info)`: repair a level
    12/14/15 stream from its intact shards.  Raises UnnecessaryScrub when the
    stream verifies.  Surviving shards are decoded with their true indices
    (the reference numbers them by position, which only works while the lost
    shards are parity shards)."""
    if len(hash) != HASH_SIZE:
        raise HashDecodeError(HASH_SIZE, len(hash))
    a = as_u8(input)
    h = as_u8(hash)
    out = OutBytes(a.size)
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_scrub(ptr(a), a.size, ptr(h), h.size, encode_info.padding_len, encode_info.chunk_len,
                                out.ptr(), a.size, ctypes.byref(olen)))
    return out.result(olen.value)
