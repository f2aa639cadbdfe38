"""Randomised parity sweep over the single-object routes.

One object's encode()/decode() (encoding.rs:86-172, decoding.rs:80-114) is
routed by size and format bits: KS zero-copy up to 64 chunks, KM (staged or
not) up to 32768, K13 beyond; the zero-copy zfec paths up to a 64 MiB pinned
footprint; the host stages straight into pinned memory.  Seeded random
(level, size) pairs — sizes drawn log-uniformly from 1 B to 6 MiB, so every
route and the boundaries between them get hit — are checked bit-exact
against the C oracle (injected ECIES key and nonce), decoded back, and, with
the Bao bit, rejected after one flipped byte; the same for zfec's stage
functions with random shapes and random erasures against the C oracle.
"""
import math
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SK = bytes(range(3, 35))
EPH = bytes(range(41, 73))
NONCE = bytes(range(9, 25))


def _size(rng):
    return max(1, int(math.exp(rng.uniform(0, math.log(6 << 20)))))


def _data(rng, n, level):
    d = np.frombuffer(rng.randbytes(n), dtype=np.uint8).copy()
    if level & 2 and rng.random() < 0.5:  # compressible for the snappy stage now and then
        d[::4] = 0x41
    return d.tobytes()


@pytest.mark.parametrize("seed", range(4))
def test_random_levels_and_sizes(gpu, seed):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    rng = random.Random(1000 + seed)
    pub = O.c_public_key(SK)
    for _ in range(16):
        level = rng.randrange(16)
        n = _size(rng)
        d = _data(rng, n, level)
        pk = pub if level & 1 else b""
        oenc, oh, oinfo = O.c_encode_full(d, level, pk, EPH, NONCE)
        enc, h, info = ca.encode(pk, d, level, ephemeral_sk=EPH, nonce=NONCE)
        assert enc == oenc, (level, n)
        assert h == oh and info.padding_len == oinfo["padding_len"], (level, n)
        assert ca.decode(SK, h, enc, info.padding_len, level) == d, (level, n)
        if level & 4 and len(enc) > 8:
            bad = bytearray(enc)
            bad[rng.randrange(8, len(bad))] ^= 1 << rng.randrange(8)
            with pytest.raises(BaoDecodeError):
                ca.decode(SK, h, bytes(bad), info.padding_len, level)


@pytest.mark.parametrize("seed", range(3))
def test_random_zfec_shapes_and_erasures(gpu, seed):
    import carbonado_amd as ca
    rng = random.Random(2000 + seed)
    for _ in range(10):
        k = rng.choice([1, 2, 3, 4, 5, 8, 11, 16])
        m = k + rng.randrange(1, min(8, 256 - k) + 1)
        n = _size(rng) // 2 + 1
        d = rng.randbytes(n)
        shards, pad, C = ca.encoding.zfec(d, k, m)
        oshards, opad, oC = O.zfec_encode(d, k, m)
        assert (shards, pad, C) == (oshards, opad, oC), (k, m, n)
        keep = sorted(rng.sample(range(m), k))
        rng.shuffle(keep)
        parts = [shards[i * C:(i + 1) * C] for i in keep]
        assert ca.decoding.zfec_chunks(parts, pad, keep, k, m) == d, (k, m, n, keep)
