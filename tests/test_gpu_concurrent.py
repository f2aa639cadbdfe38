"""Single-object encode()/decode() from many host threads at once.

A storage node calls carbonado's encode()/decode() (encoding.rs:86-172,
decoding.rs:80-114) per segment from several threads.  Each calling thread
has its own context here (HIP stream, grow-only device and pinned buffers,
KM's last-workgroup counter in its stream's queue block), and the threads
share the host stage pool (a caller that finds it busy runs its host copies
and stages alone).  Six threads run the same mix of objects, shuffled per
thread, over the KS (small), KM (single-object multi-workgroup), zero-copy
zfec and K13 (beyond KM's 32768 chunks) paths and the host stages: every
stream and hash equals the C oracle's, every decode gives the input back, and
a tampered stream is rejected with nothing returned.
"""
import random
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SK = bytes(range(1, 33))
EPH = bytes(range(101, 133))
NONCE = bytes(range(7, 23))
# (level, bytes): KS, KM at levels 12 / 4, zero-copy zfec at 8, snappy at 14,
# the full pipeline at 15, and a level-12 object past KM's limit (K13)
CASES = [(12, 5000), (12, 300_001), (12, 1 << 20), (4, 200_000), (8, 1 << 20), (14, 700_000), (15, 1 << 20),
         (12, 20 << 20)]


def _data(level, n):
    rng = np.random.default_rng(level * 1000 + n % 997)
    d = rng.integers(0, 256, n, dtype=np.uint8)
    if level & 2:  # compressible, so the snappy stage emits copies
        d[::3] = 7
    return d.tobytes()


def test_single_object_calls_from_many_threads(gpu):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    pub = O.c_public_key(SK)
    want = {}
    for level, n in CASES:
        d = _data(level, n)
        enc, h, info = O.c_encode_full(d, level, pub if level & 1 else b"", EPH, NONCE)
        want[(level, n)] = (d, enc, h, info["padding_len"])

    def worker(seed):
        order = list(CASES) * 2
        random.Random(seed).shuffle(order)
        bad = []
        for level, n in order:
            d, oenc, oh, pad = want[(level, n)]
            enc, h, info = ca.encode(pub if level & 1 else b"", d, level, ephemeral_sk=EPH, nonce=NONCE)
            if enc != oenc or (level & 4 and h != oh) or info.padding_len != pad:
                bad.append(("encode", level, n))
                continue
            if ca.decode(SK, h, enc, pad, level) != d:
                bad.append(("decode", level, n))
            if level & 4:
                t = bytearray(enc)
                t[len(t) // 3] ^= 0x10
                try:
                    ca.decode(SK, h, bytes(t), pad, level)
                    bad.append(("tamper accepted", level, n))
                except BaoDecodeError:
                    pass
        return bad

    with ThreadPoolExecutor(6) as ex:
        results = list(ex.map(worker, range(6)))
    assert all(not r for r in results), results
