"""Single-object call latency of the drop-in API (carbonado_amd.encode /
decode, one object per call, ordinary `bytes` in and out, as the crate's
encode()/decode() are called) against the C oracle on one host thread.
Calibration tool (not a test): python tools/latency_probe.py [reps] [levels,..] [sizes,..]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import carbonado_amd as ca  # noqa: E402
from oracle import host_oracle as H  # noqa: E402
from oracle import oracle as O  # noqa: E402

SK = H.sha256(b"latency receiver")
PUB = H.public_key(SK)


def med_us(f, reps):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e6


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    levels = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [12, 15, 8, 4]
    sizes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1024, 8192, 65536, 1 << 20, 16 << 20]
    rng = np.random.default_rng(7)
    print(f"{'level':>5} {'bytes':>9} {'enc_us':>9} {'dec_us':>9} {'oracle_enc_us':>13}  (median of {reps})")
    for level in levels:
        for n in sizes:
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            pk = PUB if level & 1 else b""
            sk = SK if level & 1 else b""
            enc, h, info = ca.encode(pk, data, level)
            assert ca.decode(sk, h, enc, info.padding_len, level) == data
            e = med_us(lambda: ca.encode(pk, data, level), reps)
            d = med_us(lambda: ca.decode(sk, h, enc, info.padding_len, level), reps)
            o = med_us(lambda: O.encode(data, level), max(3, reps // 4)) if not level & 3 else float("nan")
            print(f"{level:>5} {n:>9} {e:>9.1f} {d:>9.1f} {o:>13.1f}", flush=True)


if __name__ == "__main__":
    main()
