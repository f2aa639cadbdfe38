"""Device-resident batch API over torch tensors (the throughput path).

torch provides HBM allocations and the stream; every byte of work is done by
the HIP kernels behind the C-ABI batch entry points.  All functions enqueue
on torch's current stream and return without synchronising.
"""
from __future__ import annotations

import ctypes

import numpy as np

import torch

from . import _lib
from ._buf import check
from .constants import FEC_K, FEC_M


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def zfec_encode_batch(inp: torch.Tensor, n: int, out: torch.Tensor, k: int = FEC_K, m: int = FEC_M) -> None:
    """inp: uint8 [count, in_stride] (first n bytes of each row are data);
    out: uint8 [count, >= m*chunk_len]."""
    assert inp.dtype == torch.uint8 and out.dtype == torch.uint8 and inp.is_cuda and out.is_cuda
    assert inp.is_contiguous() and out.is_contiguous() and inp.shape[0] == out.shape[0]
    count = inp.shape[0]
    need = _lib.lib().chip_zfec_encoded_len(n, k, m)
    assert out.shape[1] >= need and inp.shape[1] >= n
    check(_lib.lib().chip_zfec_encode_batch_dev(k, m, _p(inp), inp.shape[1], n, count, _p(out), out.shape[1],
                                                _stream()))


def hbm_pattern_batch(inp: torch.Tensor, n: int, out: torch.Tensor, k: int = FEC_K, m: int = FEC_M) -> None:
    """Diagnostic: zfec_encode_batch's memory pattern (same loads, stores,
    grid and run queue) without the GF arithmetic — `out` receives the data
    shards and, per computed row q, their XOR with every byte XOR q; not
    parity (chip_hbm_pattern_batch_dev)."""
    assert inp.is_cuda and out.is_cuda and inp.is_contiguous() and out.is_contiguous()
    assert inp.shape[0] == out.shape[0] and inp.data_ptr() != out.data_ptr()
    need = _lib.lib().chip_zfec_encoded_len(n, k, m)
    assert out.shape[1] >= need and inp.shape[1] >= n
    check(_lib.lib().chip_hbm_pattern_batch_dev(k, m, _p(inp), inp.shape[1], n, inp.shape[0], _p(out),
                                                out.shape[1], _stream()))


def zfec_decode_batch(enc: torch.Tensor, chunk_len: int, indices, out: torch.Tensor,
                      k: int = FEC_K, m: int = FEC_M) -> None:
    """enc: uint8 [count, >= m*chunk_len] (shard i at i*chunk_len); `indices`
    lists the surviving shares; out: uint8 [count, >= k*chunk_len]."""
    assert enc.is_contiguous() and out.is_contiguous() and enc.shape[0] == out.shape[0]
    idx = list(indices)
    cidx = (ctypes.c_uint32 * len(idx))(*idx)
    check(_lib.lib().chip_zfec_decode_batch_dev(k, m, _p(enc), enc.shape[1], chunk_len, cidx, len(idx),
                                                enc.shape[0], _p(out), out.shape[1], _stream()))


_pools = {}


def batch_pool(device=None):
    """A torch MemPool whose segments come from chip_device_alloc (physically
    contiguous HBM where available), for multi-GiB batch buffers."""
    dev = torch.device(device or "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _pools:
        alloc = torch.cuda.memory.CUDAPluggableAllocator(str(_lib.LIB_PATH), "chip_torch_alloc", "chip_torch_free")
        with torch.cuda.device(idx):
            _pools[idx] = (alloc, torch.cuda.MemPool(alloc.allocator()))
    return _pools[idx][1]


def empty_batch(shape, device=None) -> torch.Tensor:
    """uint8 tensor for a batch buffer, allocated in batch_pool()."""
    dev = torch.device(device or "cuda")
    with torch.cuda.device(dev), torch.cuda.use_mem_pool(batch_pool(dev)):
        return torch.empty(shape, dtype=torch.uint8, device=dev)


def bao_scratch(n: int, count: int, device=None) -> torch.Tensor:
    size = _lib.lib().chip_bao_scratch_len(n, count)
    return torch.empty(size, dtype=torch.uint8, device=device or "cuda")


def bao_encode_batch(inp: torch.Tensor, n: int, out: torch.Tensor | None, hashes: torch.Tensor,
                     scratch: torch.Tensor, out_offset: int = 0) -> None:
    """out: uint8 [count, >= out_offset + bao_len(n)] or None (hash only), each
    stream `out_offset` bytes into its row (8-B multiple; 56: every chunk and
    node on a 64-B boundary); hashes: uint8 [count, 32]."""
    assert inp.is_contiguous() and inp.shape[1] >= n  # the row stride is inp.shape[1]
    count = inp.shape[0]
    check(_lib.lib().chip_bao_encode_batch_dev(
        _p(inp), inp.shape[1], n, count,
        ctypes.c_void_p(out.data_ptr() + out_offset) if out is not None else ctypes.c_void_p(0),
        out.shape[1] if out is not None else 0, _p(hashes), _p(scratch), _stream()))


def encode_scratch(fmt: int, n: int, count: int, device=None) -> torch.Tensor:
    size = _lib.lib().chip_encode_scratch_len(fmt, n, count)
    return torch.empty(size, dtype=torch.uint8, device=device or "cuda")


def encode_batch(fmt: int, inp: torch.Tensor, n: int, out: torch.Tensor, hashes: torch.Tensor,
                 scratch: torch.Tensor, out_offset: int = 0):
    """encode() of device-resident objects at a level without host stages
    (Bao and/or Zfec bits): inp uint8 [count, in_stride] (first n bytes of each
    row), out uint8 [count, >= out_offset + encoded length], hashes uint8
    [count, 32]; each encoding starts `out_offset` bytes into its row (56 with
    a 256-B multiple row: STREAM_OFFSET, the fast layout of Zfec|Bao streams,
    include/carbonado_hip.h).  Zfec|Bao runs fused (shards hashed on chip,
    written into their bao slots).  Returns (encoded length, EncodeInfoC)."""
    assert inp.is_cuda and out.is_cuda and inp.is_contiguous() and out.is_contiguous()
    assert inp.shape[0] == out.shape[0] == hashes.shape[0] and inp.shape[1] >= n
    olen = ctypes.c_uint64()
    info = _lib.EncodeInfoC()
    check(_lib.lib().chip_encode_batch_dev(fmt, _p(inp), inp.shape[1], n, inp.shape[0],
                                           ctypes.c_void_p(out.data_ptr() + out_offset), out.shape[1],
                                           ctypes.byref(olen), _p(hashes), ctypes.byref(info), _p(scratch),
                                           _stream()))
    assert out_offset + olen.value <= out.shape[1]
    return olen.value, info


# Where a Zfec|Bao stream starts in a row of 256-B multiple pitch for the fast
# layout: its 8-byte header fills the end of a 64-B segment, so every chunk and
# parent node after it starts on a 64-B boundary (include/carbonado_hip.h).
STREAM_OFFSET = 56


def decode_scratch(fmt: int, in_len: int, count: int, device=None) -> torch.Tensor:
    size = _lib.lib().chip_decode_scratch_len(fmt, in_len, count)
    return torch.empty(size, dtype=torch.uint8, device=device or "cuda")


def decode_batch(fmt: int, enc: torch.Tensor, in_len: int, hashes: torch.Tensor, padding: int, out: torch.Tensor,
                 status: torch.Tensor, scratch: torch.Tensor, in_offset: int = 0) -> int:
    """decode() of device-resident encodings at a level without host stages:
    enc uint8 [count, in_stride] (in_len bytes of each row from in_offset:
    STREAM_OFFSET where encode_batch put them), hashes uint8 [count, 32], out
    uint8 [count, >= decoded length], status int32 [count] (0, or the
    chip_status of that object).  Returns the decoded length."""
    assert enc.is_cuda and out.is_cuda and enc.is_contiguous() and out.is_contiguous()
    assert enc.shape[0] == out.shape[0] == status.shape[0] and enc.shape[1] >= in_offset + in_len
    olen = ctypes.c_uint64()
    check(_lib.lib().chip_decode_batch_dev(fmt, ctypes.c_void_p(enc.data_ptr() + in_offset), enc.shape[1], in_len,
                                           enc.shape[0], _p(hashes), padding,
                                           _p(out), out.shape[1], ctypes.byref(olen), _p(status), _p(scratch),
                                           _stream()))
    return olen.value


def bao_decode_batch(enc: torch.Tensor, n: int, hashes: torch.Tensor, out: torch.Tensor,
                     status: torch.Tensor, scratch: torch.Tensor, in_offset: int = 0) -> None:
    """status: int32/uint32 [count]; 0 = verified, 5 = hash mismatch.  Each
    stream `in_offset` bytes into its row of enc (8-B multiple)."""
    count = enc.shape[0]
    check(_lib.lib().chip_bao_decode_batch_dev(ctypes.c_void_p(enc.data_ptr() + in_offset), enc.shape[1], n, count,
                                               _p(hashes), _p(out), out.shape[1], _p(status), _p(scratch),
                                               _stream()))


def scrub_scratch(length: int, count: int, device=None) -> torch.Tensor:
    size = _lib.lib().chip_scrub_scratch_len(length, count)
    return torch.empty(size, dtype=torch.uint8, device=device or "cuda")


def scrub_batch(enc: torch.Tensor, length: int, hashes: torch.Tensor, padding: int, chunk_len: int,
                out: torch.Tensor, scratch: torch.Tensor, offset: int = 0) -> np.ndarray:
    """scrub() (decoding.rs:159-212) of device-resident Bao|Zfec streams
    enc uint8 [count, >= length] with one EncodeInfo; repaired streams go to
    the rows of `out`.  Returns the per-object statuses (int32 numpy):
    0 = repaired, CHIP_ERR_UNNECESSARY_SCRUB = intact, else scrub's error.
    A row of `out` is written only where the status is 0 (its repaired
    stream's hash matched); every other row is left untouched.  The streams
    sit `offset` bytes into their rows of enc and out (8-B multiple)."""
    assert enc.is_cuda and out.is_cuda and enc.is_contiguous() and out.is_contiguous()
    count = enc.shape[0]
    assert out.shape[0] == count and hashes.shape[0] == count
    status = np.zeros(count, dtype=np.int32)
    check(_lib.lib().chip_scrub_batch_dev(ctypes.c_void_p(enc.data_ptr() + offset), enc.shape[1], length, count,
                                          _p(hashes), padding, chunk_len, ctypes.c_void_p(out.data_ptr() + offset),
                                          out.shape[1], status.ctypes.data_as(ctypes.c_void_p), _p(scratch),
                                          _stream()))
    return status


def encode_host_batch(fmt: int, inp: torch.Tensor, n: int, out: torch.Tensor, hashes: torch.Tensor,
                      nslots: int = 3, slice_bytes: int = 256 << 20, pubkey: bytes = b"",
                      ephemeral_sk=None, nonce=None, host_threads: int = 0):
    """End-to-end encode() of `count` objects held in HOST memory (pinned
    tensors reach the full PCIe rate): inp uint8 [count, >= n], out uint8
    [count, >= chip_encode_max_len(n)], hashes uint8 [count, 32].  The
    Snappy/Ecies host stages of a slice run on `host_threads` threads while
    earlier slices are on the device.  `ephemeral_sk` [count, 32] / `nonce`
    [count, 16] (uint8 tensors or arrays) inject the ECIES randomness (tests).
    Synchronous.  Returns (encoded length per object, EncodeInfo per object)."""
    import numpy as np
    from .structs import EncodeInfo
    assert not inp.is_cuda and not out.is_cuda and not hashes.is_cuda
    assert inp.is_contiguous() and out.is_contiguous() and hashes.is_contiguous()
    count = inp.shape[0]
    olen = (ctypes.c_uint64 * max(count, 1))()
    info = (_lib.EncodeInfoC * max(count, 1))()
    keep = [np.ascontiguousarray(np.asarray(x, dtype=np.uint8)) if x is not None else None
            for x in (ephemeral_sk, nonce)]
    inj = None
    if any(k is not None for k in keep):
        inj = _lib.EciesInjectC(*[k.ctypes.data if k is not None else None for k in keep])
    pk = np.frombuffer(bytes(pubkey), dtype=np.uint8)
    check(_lib.lib().chip_encode_host_batch(fmt, pk.ctypes.data if pk.size else None, pk.size,
                                            ctypes.byref(inj) if inj is not None else None, _p(inp), n, count,
                                            inp.shape[1], _p(out), out.shape[1], olen, _p(hashes), info,
                                            nslots, slice_bytes, host_threads))
    # field tuples through numpy (one C-speed pass), then EncodeInfo(*t): half
    # the cost of from_c per object at 16384 objects
    rows = np.ctypeslib.as_array(info)[:count].tolist() if count else []
    return list(olen)[:count], [EncodeInfo(*r) for r in rows]


def decode_host_batch(fmt: int, enc: torch.Tensor, in_len, hashes: torch.Tensor, padding, out: torch.Tensor,
                      secret_key: bytes = b"", nslots: int = 3, slice_bytes: int = 256 << 20,
                      host_threads: int = 0, raise_first: bool = True):
    """End-to-end decode() of `count` encoded objects held in HOST memory:
    enc uint8 [count, >= max in_len], in_len / padding per object, hashes
    uint8 [count, 32], out uint8 [count, out_stride].  Synchronous.  Returns
    (decoded length per object, status per object); with raise_first the
    first failing object's status is raised as its CarbonadoError."""
    import numpy as np
    from .error import status_to_error
    assert not enc.is_cuda and not out.is_cuda and not hashes.is_cuda
    assert enc.is_contiguous() and out.is_contiguous() and hashes.is_contiguous()
    count = enc.shape[0]
    n = max(count, 1)
    lens = (ctypes.c_uint64 * n)(*[int(x) for x in in_len])
    pads = (ctypes.c_uint32 * n)(*[int(x) for x in padding])
    olen = (ctypes.c_uint64 * n)()
    st = (ctypes.c_int32 * n)()
    sk = np.frombuffer(bytes(secret_key), dtype=np.uint8)
    rc = _lib.lib().chip_decode_host_batch(fmt, sk.ctypes.data if sk.size else None, sk.size, _p(hashes), _p(enc),
                                           lens, count, enc.shape[1], pads, _p(out), out.shape[1], olen, st,
                                           nslots, slice_bytes, host_threads)
    statuses = [st[o] for o in range(count)]
    if rc and (raise_first or not any(statuses)):
        raise status_to_error(rc)
    return [olen[o] for o in range(count)], statuses


def host_topology() -> dict:
    """Where this process's host-copy path sits (chip_host_topology): the
    GPU's NUMA node, the calling thread's staging ring node and the copy
    workers' nodes (diagnostic)."""
    import json
    L = _lib.lib()
    n = ctypes.c_uint64(0)
    L.chip_host_topology(None, 0, ctypes.byref(n))
    buf = ctypes.create_string_buffer(max(1, n.value))
    check(L.chip_host_topology(buf, n.value, ctypes.byref(n)))
    return json.loads(buf.value.decode())
