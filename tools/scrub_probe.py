"""Time breakdown of scrub() on one 16 MiB object (calibration tool, not
product code): the bare C-ABI call into a reused pinned/pageable buffer vs the
Python mirror (which allocates the output and returns bytes)."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import carbonado_amd as ca  # noqa: E402
from carbonado_amd import _lib  # noqa: E402
from carbonado_amd._buf import ptr  # noqa: E402


def t(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


n = 16 << 20
d = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
enc, h, info = ca.encode(b"", d, 12)
bad = np.frombuffer(enc, np.uint8).copy()
bad[bench.scrub_corrupt_offset(n, 0)] ^= 0x40
L = _lib.lib()
hh = np.frombuffer(h, np.uint8).copy()
out = np.empty(bad.size, np.uint8)
olen = ctypes.c_uint64()
pin_in = torch.from_numpy(bad).pin_memory().numpy()
pin_out = torch.empty(bad.size, dtype=torch.uint8).pin_memory().numpy()


def raw(src, dst):
    rc = L.chip_scrub(ptr(src), src.size, ptr(hh), 32, info.padding_len, info.chunk_len, ptr(dst), dst.size,
                      ctypes.byref(olen))
    assert rc == 0, rc


print(f"python scrub():            {t(lambda: ca.decoding.scrub(bad, h, info)):8.3f} ms")
print(f"C-ABI pageable, reused out: {t(lambda: raw(bad, out)):8.3f} ms")
print(f"C-ABI pinned in/out:        {t(lambda: raw(pin_in, pin_out)):8.3f} ms")
print(f"verify (bao decode) only:   {t(lambda: ca.decode(b'', h, enc, info.padding_len, 12)):8.3f} ms")
print(f"encode() level 12:          {t(lambda: ca.encode(b'', d, 12)):8.3f} ms")
print(f"np.empty+tobytes 32 MiB:    {t(lambda: np.empty(bad.size, np.uint8).tobytes()):8.3f} ms")
assert bytes(out[:olen.value]) == enc
print("ok")

# distinct inputs per object (the bench's working set)
objs = []
for i in range(16):
    di = np.random.default_rng(100 + i).integers(0, 256, n, dtype=np.uint8)
    e, hi, inf = ca.encode(b"", di, 12)
    b = np.frombuffer(e, np.uint8).copy()
    b[bench.scrub_corrupt_offset(n, i)] ^= 0x40
    objs.append((b, hi, inf))
held = [None] * 16


def np_scrub(b, hi, inf, shift=None):
    o = np.empty(b.size + 8192, np.uint8)
    if shift is not None:  # place the destination at page offset `shift`
        a = o.ctypes.data
        k = (shift - a) % 4096
        o = o[k:k + b.size]
    else:
        o = o[:b.size]
    hh2 = np.frombuffer(hi, np.uint8)
    rc = L.chip_scrub(ptr(b), b.size, ptr(hh2), 32, inf.padding_len, inf.chunk_len, ptr(o), o.size,
                      ctypes.byref(olen))
    assert rc == 0
    return o[:olen.value].tobytes()


for name, fn, keep in (("distinct OutBytes retained", ca.decoding.scrub, True),
                       ("distinct numpy retained", np_scrub, True),
                       ("distinct numpy @page+0", lambda *a: np_scrub(*a, shift=0), True),
                       ("distinct numpy @page+48", lambda *a: np_scrub(*a, shift=48), True),
                       ("distinct numpy @page+64", lambda *a: np_scrub(*a, shift=64), True),
                       ("distinct numpy @page+4", lambda *a: np_scrub(*a, shift=4), True),
                       ("distinct OutBytes dropped", ca.decoding.scrub, False)):
    ts = []
    for p in range(3):
        for i in range(16):
            t0 = time.perf_counter()
            r = fn(*objs[i])
            if keep:
                held[i] = r
            del r
            ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{name:28s} median {ts[len(ts) // 2] * 1e3:8.3f} ms  max {ts[-1] * 1e3:8.3f} ms")
