"""GPU parity of KS, the single-launch path for single small objects
(carbonado_amd/csrc/small_kernels.hip: bao streams of N <= 512 chunks, four
lanes per BLAKE3 compression).  Every size class around its limits — empty
input, partial chunks and blocks, N = 1 (the chunk is the root), N = 2,
odd and power-of-two chunk counts, the N = 512 / 513 border with the batch
kernels — bit-exact against the C oracle; decode rejects a flipped byte in
the header, a chunk, a parent node and the hash (the same cases
test_gpu_bao.py holds for the batch kernels)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

BAO_SIZES = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 3 * 1024 + 7, 8192, 65536 - 5, 100_000,
             511 * 1024 + 1, 512 * 1024, 512 * 1024 + 1]
# encode() level 12: N = 8 C / 1024, C = ceil(n / 4096) * 1024: N = 8 .. 512 and 520
ZFEC_SIZES = [0, 1, 4095, 4096, 4097, 10_000, 65536, 64 * 4096 - 3, 64 * 4096, 64 * 4096 + 1]


def _data(n, seed=0):
    return np.random.default_rng(n * 7 + seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n", BAO_SIZES)
def test_small_bao_encode_decode(gpu, n):
    import carbonado_amd as ca
    d = _data(n)
    enc, h = ca.encoding.bao(d)
    oenc, oh = O.bao_encode(d)
    assert h == oh and enc == oenc
    assert ca.encoding.blake3(d) == oh  # hash-only call (no stream buffer)
    assert ca.decoding.bao(enc, h) == d


@pytest.mark.parametrize("n", ZFEC_SIZES)
@pytest.mark.parametrize("level", [4, 12])
def test_small_encode_levels(gpu, n, level):
    import carbonado_amd as ca
    d = _data(n, level)
    enc, h, info = ca.encode(b"", d, level)
    oenc, oh, _ = O.encode(d, level)
    assert h == oh and enc == oenc
    assert ca.decode(b"", h, enc, info.padding_len, level) == d


@pytest.mark.parametrize("n", [1, 1024, 3000, 70_000])
def test_small_decode_rejects_tampering(gpu, n):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    d = _data(n, 3)
    enc, h = ca.encoding.bao(d)
    N = max(1, (n + 1023) // 1024)
    spots = [8, len(enc) - 1]  # first content (or parent) byte, last byte
    if N > 1:
        spots.append(8 + 64 + 5)  # inside the first chunk (after the root's node)
    for pos in spots:
        bad = bytearray(enc)
        bad[pos] ^= 0x10
        with pytest.raises(BaoDecodeError):
            ca.decoding.bao(bytes(bad), h)
    bad_h = bytearray(h)
    bad_h[31] ^= 1
    with pytest.raises(BaoDecodeError):
        ca.decoding.bao(enc, bytes(bad_h))


def test_small_level12_decode_rejects_parent_flip(gpu):
    """A parent node of the Zfec|Bao stream (not only content) is checked."""
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    d = _data(20_000, 5)
    enc, h, info = ca.encode(b"", d, 12)
    bad = bytearray(enc)
    bad[8 + 3] ^= 0x80  # the root's node (left CV)
    with pytest.raises(BaoDecodeError):
        ca.decode(b"", h, bytes(bad), info.padding_len, 12)
    assert ca.decode(b"", h, enc, info.padding_len, 12) == d


def test_small_matches_batch_kernels(gpu):
    """The same objects through KS (one object per call) and the batch
    kernels (a device batch of several objects): identical streams and hashes."""
    import torch
    import carbonado_amd as ca
    from carbonado_amd import device as D
    n, count = 37_000, 3
    objs = [_data(n, s) for s in range(count)]
    stride = (n + 15) // 16 * 16
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for i, o in enumerate(objs):
        inp[i, :n] = torch.frombuffer(bytearray(o), dtype=torch.uint8).cuda()
    for level in (4, 12):
        single = [ca.encode(b"", o, level) for o in objs]
        olen = len(single[0][0])
        ostride = (olen + 15) // 16 * 16
        out = torch.zeros((count, ostride), dtype=torch.uint8, device="cuda")
        hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
        D.encode_batch(level, inp, n, out, hashes, D.encode_scratch(level, n, count))
        torch.cuda.synchronize()
        for i in range(count):
            assert bytes(out[i, :olen].cpu().numpy()) == single[i][0]
            assert bytes(hashes[i].cpu().numpy()) == single[i][1]


# batches of tiny objects (bao stream of at most 64 chunks): one 64-thread
# workgroup per object; n values give N = 1, 2, 7, 63, 64 (and 65 / 72: the
# batch kernels) at level 4, N = 8, 16, 64 (and 72) at level 12
TINY = [(4, 0), (4, 1), (4, 1025), (4, 6 * 1024 + 1), (4, 63 * 1024), (4, 64 * 1024), (4, 64 * 1024 + 1),
        (12, 1), (12, 4097), (12, 32768), (12, 32769)]


@pytest.mark.parametrize("level,n", TINY)
def test_tiny_batches(gpu, level, n):
    import torch
    from carbonado_amd import device as D
    count = 9
    objs = [_data(n, 40 + s) for s in range(count)]
    stride = max(16, (n + 15) // 16 * 16)
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for i, o in enumerate(objs):
        if n:
            inp[i, :n] = torch.frombuffer(bytearray(o), dtype=torch.uint8).cuda()
    oenc, oh, oinfo = O.encode(objs[0], level)
    olen = len(oenc)
    ostride = (olen + 15) // 16 * 16
    out = torch.zeros((count, ostride), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    got_len, info = D.encode_batch(level, inp, n, out, hashes, D.encode_scratch(level, n, count))
    torch.cuda.synchronize()
    assert got_len == olen
    encs = []
    for i in range(count):
        e, h, _ = O.encode(objs[i], level)
        assert bytes(out[i, :olen].cpu().numpy()) == e, i
        assert bytes(hashes[i].cpu().numpy()) == h, i
        encs.append(e)
    # decode the batch back; object 4's stream has one flipped byte
    bad = out.clone()
    bad[4, olen - 1] ^= 1
    dec = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    D.decode_batch(level, bad, olen, hashes, info.padding_len, dec, status,
                   D.decode_scratch(level, olen, count))
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    assert st[4] == 5 and all(s == 0 for i, s in enumerate(st) if i != 4), st
    for i in range(count):
        if i != 4:
            assert bytes(dec[i, :n].cpu().numpy()) == objs[i], i


@pytest.mark.parametrize("seed", range(12))
def test_tiny_batches_randomized(gpu, seed):
    """Seeded random batches for the tiny-object path (several objects per
    workgroup when N <= 8, one per workgroup up to N = 64, the batch kernels
    above): random sizes, counts, levels and a random set of tampered
    objects; every object's encoding against the oracle, every decode status
    and the intact objects' bytes."""
    import torch
    from carbonado_amd import device as D
    rng = np.random.default_rng(1000 + seed)
    level = int(rng.choice([4, 12]))
    n = int(rng.integers(0, (66 if level == 4 else 34) * 1024))
    count = int(rng.integers(2, 41))
    objs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for _ in range(count)]
    stride = max(16, (n + 15) // 16 * 16)
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for i, o in enumerate(objs):
        if n:
            inp[i, :n] = torch.frombuffer(bytearray(o), dtype=torch.uint8).cuda()
    oenc0 = O.encode(objs[0], level)[0]
    olen = len(oenc0)
    out = torch.zeros((count, (olen + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    _, info = D.encode_batch(level, inp, n, out, hashes, D.encode_scratch(level, n, count))
    torch.cuda.synchronize()
    for i in sorted({0, count - 1, int(rng.integers(0, count))}):
        e, h, _ = O.encode(objs[i], level)
        assert bytes(out[i, :olen].cpu().numpy()) == e and bytes(hashes[i].cpu().numpy()) == h, (n, count, i)
    bad = out.clone()
    hit = sorted(set(rng.integers(0, count, int(rng.integers(0, 4))).tolist()))
    for i in hit:
        bad[i, int(rng.integers(0, olen))] ^= int(rng.integers(1, 256))
    dec = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    D.decode_batch(level, bad, olen, hashes, info.padding_len, dec, status, D.decode_scratch(level, olen, count))
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    for i in range(count):
        assert st[i] == (5 if i in hit else 0), (n, count, i, st[i])
        if i not in hit:
            assert bytes(dec[i, :n].cpu().numpy()) == objs[i], (n, count, i)


_K13_C1024 = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import carbonado_amd as ca
from carbonado_amd import device as D
from oracle import oracle as O
ca._lib.lib().chip_init(0)
bad = []
for n in (1, 1000, 4095, 4096):
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    oenc, oh, _ = O.encode(d, 12)
    enc, h, info = ca.encode(b"", d, 12)
    if enc != oenc or h != oh:
        bad.append(("single", n))
    # a device batch of 3 objects (count >= 2 also takes K13 with KS off)
    count, stride = 3, max(16, (n + 15) // 16 * 16)
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for i in range(count):
        inp[i, :n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    out = torch.zeros((count, (len(oenc) + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    D.encode_batch(12, inp, n, out, hashes, D.encode_scratch(12, n, count))
    torch.cuda.synchronize()
    for i in range(count):
        if bytes(out[i, :len(oenc)].cpu().numpy()) != oenc or bytes(hashes[i].cpu().numpy()) != oh:
            bad.append(("batch", n, i))
print("BAD", bad) if bad else print("OK")
"""


def test_k13_one_column_shards_with_ks_off(gpu, tmp_path):
    """K13's general path at C == 1024 (N == 8: the whole tree
    lies in levels 1-3) must finalize the root itself.  KS normally takes
    these objects, so the run switches it off (CHIP_SMALL=0, read once per
    process) in a child process and compares streams and hashes with the
    oracle, single objects and a device batch."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    env = dict(os.environ, CHIP_SMALL="0")
    out = subprocess.run([sys.executable, "-c", _K13_C1024, root], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK"), out.stdout + out.stderr
