"""Host-stage capacity on this machine: T threads each running snap+ecies
(encode direction) or ecies-decrypt+unsnap (decode direction) on 16 MiB
random objects through the C-ABI (ctypes releases the GIL).  Calibration
tool for the level-15 end-to-end pipeline."""
import ctypes
import sys
import threading
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import carbonado_amd as ca  # noqa: E402
from carbonado_amd import _lib  # noqa: E402

L = _lib.lib()
n = 16 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
sk = bytes([7] * 32)
pub = ca.encoding.public_key(sk)
src = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
frame = np.frombuffer(ca.encoding.snap(src.tobytes()), np.uint8).copy()
env = np.frombuffer(ca.encoding.ecies(pub, frame.tobytes()), np.uint8).copy()


def enc_worker(res):
    f = np.zeros(frame.size + 64, np.uint8)
    e = np.zeros(env.size + 64, np.uint8)
    ol = ctypes.c_uint64()
    t0 = time.perf_counter()
    for _ in range(reps):
        L.chip_snap_compress(src.ctypes.data, n, f.ctypes.data, f.size, ctypes.byref(ol))
        L.chip_ecies_encrypt(pub, 65, None, f.ctypes.data, ol.value, e.ctypes.data, e.size, ctypes.byref(ol))
    res.append(time.perf_counter() - t0)


def dec_worker(res):
    d = np.zeros(env.size, np.uint8)
    u = np.zeros(n + 64, np.uint8)
    ol = ctypes.c_uint64()
    t0 = time.perf_counter()
    for _ in range(reps):
        L.chip_ecies_decrypt(sk, 32, env.ctypes.data, env.size, d.ctypes.data, d.size, ctypes.byref(ol))
        L.chip_snap_decompress(d.ctypes.data, ol.value, u.ctypes.data, u.size, ctypes.byref(ol))
    res.append(time.perf_counter() - t0)


for T in [1, int(sys.argv[1]) if len(sys.argv) > 1 else 16]:
    for name, fn in (("encode snap+ecies", enc_worker), ("decode ecies+unsnap", dec_worker)):
        res = []
        ths = [threading.Thread(target=fn, args=(res,)) for _ in range(T)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        wall = time.perf_counter() - t0
        print(f"{name:22s} threads {T:3d}: {T * reps * n / wall / 2**30:6.2f} GiB/s aggregate "
              f"({reps * n / max(res) / 2**30:.2f} GiB/s slowest thread)", flush=True)
