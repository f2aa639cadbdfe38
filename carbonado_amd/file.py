"""file (mirror of /root/reference/src/file.rs): the 160-byte signed Header
and file::encode / file::decode through libcarbonado_hip (file_container.cpp:
the header and its BIP-340 signature on the host, the body through encode()/
decode() with zfec + bao on the MI355X)."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._buf import OutBytes, as_u8, check, ptr  # noqa: F401
from .constants import Format
from .encoding import _inject
from .structs import EncodeInfo

HEADER_LEN = 160  # file.rs:257-259 Header::len()
MAGICNO = b"CARBONADO01\n"  # constants.rs:4


def _opt(b: bytes | None, n: int):
    if b is None:
        return None, None
    a = as_u8(b)
    if a.size != n:
        raise ValueError(f"expected {n} bytes")
    return ptr(a), a


@dataclass
class Header:
    """file.rs:24-43 `pub struct Header`."""

    pubkey: bytes          # 33 bytes, compressed
    hash: bytes            # 32 bytes, bao hash
    signature: bytes       # 64 bytes, BIP-340 over `hash`
    format: Format
    chunk_index: int
    encoded_len: int
    padding_len: int
    metadata: bytes | None  # 8 bytes or None

    @staticmethod
    def len() -> int:
        return HEADER_LEN

    @classmethod
    def _from_c(cls, h: _lib.HeaderC) -> "Header":
        return cls(bytes(h.pubkey), bytes(h.hash), bytes(h.signature), Format(h.format), h.chunk_index,
                   h.encoded_len, h.padding_len, bytes(h.metadata) if h.has_metadata else None)

    def _to_c(self) -> _lib.HeaderC:
        h = _lib.HeaderC()
        ctypes.memmove(h.pubkey, self.pubkey, 33)
        ctypes.memmove(h.hash, self.hash, 32)
        ctypes.memmove(h.signature, self.signature, 64)
        h.format, h.chunk_index = int(self.format), self.chunk_index
        h.encoded_len, h.padding_len = self.encoded_len, self.padding_len
        if self.metadata is not None:
            ctypes.memmove(h.metadata, self.metadata, 8)
            h.has_metadata = 1
        return h

    @classmethod
    def new(cls, sk: bytes, pk: bytes, hash: bytes, format: int, chunk_index: int, encoded_len: int,
            padding_len: int, metadata: bytes | None, *, aux_rand: bytes | None = None) -> "Header":
        """file.rs:263-289 Header::new: signs `hash` with `sk` (BIP-340);
        `aux_rand` injects the signature's auxiliary randomness (tests)."""
        s, p, hh = as_u8(sk), as_u8(pk), as_u8(hash)
        mp, _m = _opt(metadata, 8)
        ap, _a = _opt(aux_rand, 32)
        out = _lib.HeaderC()
        check(_lib.lib().chip_header_new(ptr(s), s.size, ptr(p), p.size, ptr(hh), hh.size, int(format), chunk_index,
                                         encoded_len, padding_len, mp, ap, ctypes.byref(out)))
        return cls._from_c(out)

    def try_to_vec(self) -> bytes:
        """file.rs:292-335 Header::try_to_vec."""
        out = np.empty(HEADER_LEN, dtype=np.uint8)
        h = self._to_c()
        check(_lib.lib().chip_header_to_bytes(ctypes.byref(h), ptr(out)))
        return out.tobytes()

    @classmethod
    def try_from(cls, data) -> "Header":
        """file.rs:116-154 TryFrom<&[u8]>: magic, pubkey and signature checked."""
        a = as_u8(data)
        out = _lib.HeaderC()
        check(_lib.lib().chip_header_parse(ptr(a), a.size, ctypes.byref(out)))
        return cls._from_c(out)

    @classmethod
    def from_file(cls, path) -> "Header":
        """file.rs:45-113 TryFrom<&File>: the first 160 bytes of the file."""
        with open(path, "rb") as f:
            return cls.try_from(f.read(HEADER_LEN))

    def file_name(self) -> str:
        """file.rs:338-342: `{hex hash}.c{format}`."""
        return f"{self.hash.hex()}.c{int(self.format)}"


def encode(sk: bytes, pk: bytes | None, input, level: int, metadata: bytes | None = None, *,
           ephemeral_sk: bytes | None = None, nonce: bytes | None = None,
           aux_rand: bytes | None = None) -> tuple[bytes, EncodeInfo]:
    """file.rs:409-440 file::encode -> (header || encoded, EncodeInfo)."""
    L = _lib.lib()
    s = as_u8(sk)
    p = as_u8(pk) if pk is not None else None
    a = as_u8(input)
    mp, _m = _opt(metadata, 8)
    ap, _a = _opt(aux_rand, 32)
    inj, _keep = _inject(ephemeral_sk, nonce)
    cap = HEADER_LEN + L.chip_encode_max_len(a.size)
    out = OutBytes(cap)
    olen = ctypes.c_uint64()
    info = _lib.EncodeInfoC()
    check(L.chip_file_encode(ptr(s), s.size, ptr(p) if p is not None else None, p.size if p is not None else 0,
                             ptr(a), a.size, int(level), mp, ctypes.byref(inj) if inj is not None else None, ap,
                             out.ptr(), cap, ctypes.byref(olen), ctypes.byref(info)))
    return out.result(olen.value), EncodeInfo.from_c(info)


def decode(secret_key: bytes, encoded) -> tuple[Header, bytes]:
    """file.rs:395-407 file::decode -> (Header, decoded bytes)."""
    from .decoding import _grow_call, decoded_cap
    L = _lib.lib()
    s = as_u8(secret_key)
    a = as_u8(encoded)
    hdr = _lib.HeaderC()
    cap = 0
    if a.size >= HEADER_LEN:  # size the output from the (not yet verified) header fields
        cap = decoded_cap(a[HEADER_LEN:], int.from_bytes(a[147:151].tobytes(), "little"), Format(int(a[141]) & 15))
    body = _grow_call(lambda out, c, olen: L.chip_file_decode(ptr(s) if s.size else None, s.size, ptr(a), a.size,
                                                               ctypes.byref(hdr), out, c, ctypes.byref(olen)), cap)
    return Header._from_c(hdr), body


def _host_buffer(shape):
    """Pinned host memory for the PCIe stages (page-locked only where a device
    exists; without one the device stage fails anyway)."""
    import torch
    return torch.empty(shape, dtype=torch.uint8, pin_memory=torch.cuda.is_available())


def encode_files(in_paths, out_dir, sk: bytes, level: int, *, pk: bytes | None = None,
                 metadata: bytes | None = None, slice_objects: int = 64, host_threads: int = 16,
                 nslots: int = 3, io_threads: int = 16, fsync: bool = False, stats: dict | None = None) -> list:
    """file::encode (file.rs:409-440) over many flat files of one size, end to
    end: disk -> pinned host memory -> HBM (zfec + bao on the device, host
    Snappy/Ecies on `host_threads` threads) -> pinned host memory -> header +
    body written to `out_dir/<hash>.c<level>`.  Three stages overlap: a reader
    thread fills the next slice of `slice_objects` files while the device
    works on the current one and a writer thread signs and writes the
    previous one; each of those stages spreads its files over `io_threads`
    threads.  Returns [(output path, EncodeInfo)] in input order; `stats`
    (optional) receives the busy seconds of each stage."""
    import os
    import queue
    import threading
    import time
    from concurrent.futures import ThreadPoolExecutor
    from pathlib import Path

    import torch

    from . import device

    in_paths = [Path(p) for p in in_paths]
    out_dir = Path(out_dir)
    if not in_paths:
        return []
    n = in_paths[0].stat().st_size
    if any(p.stat().st_size != n for p in in_paths):
        raise ValueError("encode_files: every input file must have the same size (use file.encode per file)")
    L = _lib.lib()
    s = as_u8(sk)
    if pk is None:
        from .encoding import public_key
        pk = public_key(sk)
    pk = bytes(pk)
    pub33 = Header.new(sk, pk, bytes(32), 0, 0, 0, 0, None).pubkey  # the stored (compressed) form
    cap = L.chip_encode_max_len(n)
    S = max(1, min(slice_objects, len(in_paths)))
    nbuf = 2
    h_in = [_host_buffer((S, max(n, 1))) for _ in range(nbuf)]
    h_out = [_host_buffer((S, cap)) for _ in range(nbuf)]
    h_hash = [_host_buffer((S, 32)) for _ in range(nbuf)]
    slices = [list(range(i, min(i + S, len(in_paths)))) for i in range(0, len(in_paths), S)]
    results: list = [None] * len(in_paths)
    free_in, ready_in = queue.Queue(), queue.Queue()
    free_out, ready_out = queue.Queue(), queue.Queue()
    for b in range(nbuf):
        free_in.put(b)
        free_out.put(b)
    errors = []
    # Any stage that fails sets `stop`; every wait below is a timed get that
    # gives up once `stop` is set, so no stage can wait forever on a buffer a
    # failed stage will never hand back.
    stop = threading.Event()

    def fail(e):
        errors.append(e)
        stop.set()

    def get(q):
        while True:
            try:
                return q.get(timeout=0.05)
            except queue.Empty:
                if stop.is_set():
                    return None

    rpool, wpool = ThreadPoolExecutor(io_threads), ThreadPoolExecutor(io_threads)
    busy = {"read_s": 0.0, "device_s": 0.0, "write_s": 0.0}

    def read_one(buf, j, o):
        with open(in_paths[o], "rb", buffering=0) as f:
            mv = memoryview(buf[j, :n])
            got = 0
            while got < n:
                r = f.readinto(mv[got:])
                if not r:
                    raise IOError(f"short read: {in_paths[o]}")
                got += r

    def write_one(out, hashes, olens, infos, j, o):
        hdr = Header.new(sk, pub33, hashes[j].tobytes(), level, 0, infos[j].output_len, infos[j].padding_len,
                         metadata)
        path = out_dir / hdr.file_name()
        with open(path, "wb", buffering=0) as f:
            f.write(hdr.try_to_vec())
            f.write(memoryview(out[j, :olens[j]]))
            if fsync:
                os.fsync(f.fileno())
        results[o] = (path, infos[j])

    def reader():
        try:
            for sl in slices:
                b = get(free_in)
                if b is None:
                    return
                t0 = time.perf_counter()
                buf = h_in[b].numpy()
                for fut in [rpool.submit(read_one, buf, j, o) for j, o in enumerate(sl)]:
                    fut.result()
                busy["read_s"] += time.perf_counter() - t0
                ready_in.put((b, sl))
        except BaseException as e:  # noqa: BLE001
            fail(e)
        finally:
            ready_in.put(None)

    def writer():
        while True:
            item = get(ready_out)
            if item is None:  # end of the batch, or a stage failed
                return
            b, sl, olens, infos = item
            try:
                if not stop.is_set():
                    t0 = time.perf_counter()
                    out, hashes = h_out[b].numpy(), h_hash[b].numpy()
                    for fut in [wpool.submit(write_one, out, hashes, olens, infos, j, o) for j, o in enumerate(sl)]:
                        fut.result()
                    busy["write_s"] += time.perf_counter() - t0
            except BaseException as e:  # noqa: BLE001
                fail(e)
            finally:
                free_out.put(b)  # always returned, also while draining after a failure

    tr, tw = threading.Thread(target=reader), threading.Thread(target=writer)
    tr.start()
    tw.start()
    try:
        for _ in slices:
            item = None if stop.is_set() else get(ready_in)
            if item is None:
                break
            b, sl = item
            ob = get(free_out)
            if ob is None:
                break
            cnt = len(sl)
            t0 = time.perf_counter()
            try:
                olens, infos = device.encode_host_batch(level, h_in[b][:cnt], n, h_out[ob][:cnt], h_hash[ob][:cnt],
                                                        nslots, pubkey=pk, host_threads=host_threads)
            except BaseException as e:  # noqa: BLE001
                fail(e)
                break
            busy["device_s"] += time.perf_counter() - t0
            free_in.put(b)
            ready_out.put((ob, sl, olens, infos))
    finally:
        ready_out.put(None)
        if errors:
            stop.set()
        tw.join()
        stop.set()  # the writer has finished: release a reader still waiting for a buffer
        tr.join()
        rpool.shutdown()
        wpool.shutdown()
    if errors:
        raise errors[0]
    if stats is not None:
        stats.update({k: round(v, 4) for k, v in busy.items()})
    return results
