"""GPU parity of KM (carbonado_amd/csrc/multi_kernels.hip, api_single.cpp):
one object's encode()/decode() over many workgroups (a quad of lanes per
compression, a 64-chunk subtree per workgroup, the last workgroup walks the
tree top) with the split copies (the host writes the chunks it holds, gathers
the content it returns).

Bit-exact against the C oracle at every size class around KM's limits —
N = 65 (the first KM stream), odd chunk counts, the level-15 shard length of a
1 MiB segment (C = 257 KiB: shards not aligned to the 64-chunk groups),
1 MiB, 4 MiB, N = KM_MAX_N (32768) and one past it (K13 again) — for
encode() at Zfec|Bao (level 12) and Bao (level 4) and the stage functions;
decode rejects a flipped byte in the header, a data chunk, a parity chunk, a
node in the data region, a node in the tree top (above the groups) and the
hash (decoding.rs:53-60: bao's HashMismatch), and returns nothing then."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# encode() level 12: N = 8 C / 1024, C = ceil(n / 4096) KiB
L12 = [32769, 36864 + 1, 65536, 100_000, 1 << 20, (1 << 20) + 1, 1048811, 3 * (1 << 20) + 12345, 4 << 20,
       16 << 20, (16 << 20) + 1]
# bao of the content (level 4): N = ceil(n / 1024)
L4 = [65537, 66560, 100_000, 1 << 20, (4 << 20) + 3, 32 << 20, (32 << 20) + 1]


def _data(n, seed=0):
    return np.random.default_rng(n * 11 + seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n", L12)
def test_km_level12_encode_decode(gpu, n):
    import carbonado_amd as ca
    d = _data(n)
    enc, h, info = ca.encode(b"", d, 12)
    oenc, oh, _ = O.encode(d, 12)
    assert h == oh
    assert enc == oenc
    assert ca.decode(b"", h, enc, info.padding_len, 12) == d


@pytest.mark.parametrize("n", L4)
def test_km_level4_and_stage_functions(gpu, n):
    import carbonado_amd as ca
    d = _data(n, 4)
    oenc, oh = O.bao_encode(d)
    enc, h, info = ca.encode(b"", d, 4)
    assert h == oh and enc == oenc
    assert ca.decode(b"", h, enc, 0, 4) == d
    senc, sh = ca.encoding.bao(d)  # chip_bao_encode / chip_bao_decode
    assert sh == oh and senc == oenc
    assert ca.decoding.bao(senc, sh) == d


def _spots(enc, n_content):
    """Byte offsets to flip: the header, the root node, a data chunk, the last
    (parity) chunk, a node of the first group's subtree and a node above the
    groups."""
    N = (n_content + 1023) // 1024
    root = 8
    spots = {"header": 0, "root_node": root + 40, "last_chunk": len(enc) - 1}
    # chunk 0 sits after the left spine of parents: 8 + 64 * depth
    depth = (N - 1).bit_length()
    spots["chunk0"] = 8 + 64 * depth + 100
    # the parent of chunks 0-1 is the last node of the spine, level 1 (in group 0)
    spots["group0_node"] = 8 + 64 * (depth - 1) + 3
    # a level-7+ node: the spine's second node when the tree has > 7 levels
    if depth > 7:
        spots["top_node"] = 8 + 64 + 17
    return spots


@pytest.mark.parametrize("n", [100_000, 1 << 20, 1048811])
def test_km_level12_decode_rejects_tampering(gpu, n):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    d = _data(n, 7)
    enc, h, info = ca.encode(b"", d, 12)
    for name, pos in _spots(enc, info.bytes_ecc).items():
        bad = bytearray(enc)
        bad[pos] ^= 0x04
        with pytest.raises(BaoDecodeError):
            ca.decode(b"", h, bytes(bad), info.padding_len, 12)
    bad_h = bytearray(h)
    bad_h[0] ^= 1
    with pytest.raises(BaoDecodeError):
        ca.decode(b"", bytes(bad_h), enc, info.padding_len, 12)
    assert ca.decode(b"", h, enc, info.padding_len, 12) == d


@pytest.mark.parametrize("n", [65537, 1 << 20])
def test_km_bao_decode_rejects_tampering(gpu, n):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    d = _data(n, 9)
    enc, h = ca.encoding.bao(d)
    for name, pos in _spots(enc, n).items():
        bad = bytearray(enc)
        bad[pos] ^= 0x80
        with pytest.raises(BaoDecodeError):
            ca.decoding.bao(bytes(bad), h)


def test_km_matches_the_batch_kernels(gpu):
    """The same objects as single calls (KM) and as a device batch (K13 /
    K1 + K3): identical streams and hashes at levels 4 and 12."""
    import torch
    import carbonado_amd as ca
    from carbonado_amd import device as D
    n, count = 300_001, 3
    objs = [_data(n, s) for s in range(count)]
    stride = (n + 255) // 256 * 256
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    for i, o in enumerate(objs):
        inp[i, :n] = torch.frombuffer(bytearray(o), dtype=torch.uint8).cuda()
    for level in (4, 12):
        single = [ca.encode(b"", o, level) for o in objs]
        olen = len(single[0][0])
        out = torch.zeros((count, (olen + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
        hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
        D.encode_batch(level, inp, n, out, hashes, D.encode_scratch(level, n, count))
        torch.cuda.synchronize()
        for i in range(count):
            assert bytes(out[i, :olen].cpu().numpy()) == single[i][0]
            assert bytes(hashes[i].cpu().numpy()) == single[i][1]


def test_km_back_to_back_calls_reuse_the_counter(gpu):
    """KM's last-workgroup counter lives in the stream's queue block and is
    reset by each launch's last workgroup: many calls of different sizes in a
    row (and an interleaved failing decode) all give the oracle's bytes."""
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    for i, n in enumerate([70_000, 1 << 20, 200_000, 65537, 3 << 20, 100_003] * 2):
        d = _data(n, 100 + i)
        level = 12 if i % 2 == 0 else 4
        enc, h, info = ca.encode(b"", d, level)
        oenc, oh, _ = O.encode(d, level)
        assert enc == oenc and h == oh, (i, n)
        bad = bytearray(enc)
        bad[len(enc) // 3] ^= 1
        with pytest.raises(BaoDecodeError):
            ca.decode(b"", h, bytes(bad), info.padding_len, level)
        assert ca.decode(b"", h, enc, info.padding_len, level) == d


_SG_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import carbonado_amd as ca
from carbonado_amd.error import BaoDecodeError
from oracle import oracle as O
ca._lib.lib().chip_init(0)
bad = []
for n, level in ((1, 12), (5000, 12), (100_000, 12), (1 << 20, 12), (1048811, 12), (1, 4), (5000, 4), (65536, 4),
                 (65537, 4), (300_001, 4), (5 << 20, 4)):
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, h, info = ca.encode(b"", d, level)
    oenc, oh, _ = O.encode(d, level)
    if enc != oenc or h != oh:
        bad.append(("encode", n, level))
    if ca.decode(b"", h, enc, info.padding_len, level) != d:
        bad.append(("decode", n, level))
    t = bytearray(enc)
    t[len(enc) // 2] ^= 8
    try:
        ca.decode(b"", h, bytes(t), info.padding_len, level)
        bad.append(("tamper accepted", n, level))
    except BaoDecodeError:
        pass
print("BAD", bad) if bad else print("OK")
"""


@pytest.mark.parametrize("env", [{"CHIP_KM_SG": "16"}, {"CHIP_KM_SG": "32"}, {"CHIP_KM_STAGE": "0"}, {"CHIP_KM": "0"}],
                         ids=["sg16", "sg32", "unstaged", "km_off"])
def test_km_smaller_groups(gpu, env):
    """KM with 16 / 32 chunks per workgroup (CHIP_KM_SG, read once per
    process: a child process): the group levels stop lower and the top walk
    starts lower; and km_kernel where km_staged_kernel runs by default
    (CHIP_KM_STAGE=0: decode and bao of the content with each quad loading
    its chunk itself); and with CHIP_KM=0 the staged device paths of round 5
    for every size (KS and K13 through HBM buffers).  Small objects (N <= 64:
    KS zero-copy by default) and both sides of N = 64 too.  Same bytes, same
    verdicts."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    out = subprocess.run([sys.executable, "-c", _SG_CHILD, root], env=dict(os.environ, **env),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and out.stdout.strip().endswith("OK"), out.stdout + out.stderr


# zero-copy single-object zfec (api_single.cpp: single_zfec_encode_zc /
# single_zfec_decode_zc) up to a pinned footprint of ZC_MAX_BYTES = 64 MiB,
# the staged copies past it: the same bytes on both sides of the cap
ZC = [1, 4095, 65536 + 17, 1 << 20, (8 << 20) - 3, 8 << 20, (8 << 20) + 1, 40 << 20]


@pytest.mark.parametrize("n", ZC)
def test_zero_copy_zfec_both_sides_of_the_cap(gpu, n):
    import carbonado_amd as ca
    d = _data(n, 21)
    oshards, opad, oC = O.zfec_encode(d)
    shards, pad, C = ca.encoding.zfec(d)
    assert (shards, pad, C) == (oshards, opad, oC)
    enc, h, info = ca.encode(b"", d, 8)  # encode() at Zfec alone
    assert enc == oshards and info.padding_len == opad
    assert ca.decoding.zfec(shards, pad) == d
    assert ca.decode(b"", h, enc, pad, 8) == d
    # two data shards lost: the decode kernel computes them from parity
    keep = [2, 3, 5, 7]
    parts = [shards[i * C:(i + 1) * C] for i in keep]
    assert ca.decoding.zfec_chunks(parts, pad, keep) == d


@pytest.mark.parametrize("k,m,lost", [(2, 3, [0]), (8, 16, [0, 1, 2, 3, 4, 5, 6, 7]), (11, 13, [0, 4]), (16, 20, [3, 9, 15])])
def test_zero_copy_zfec_other_shapes(gpu, k, m, lost):
    import carbonado_amd as ca
    n = 300_001
    d = _data(n, k * 100 + m)
    shards, pad, C = ca.encoding.zfec(d, k, m)
    oshards, opad, oC = O.zfec_encode(d, k, m)
    assert (shards, pad, C) == (oshards, opad, oC)
    keep = [i for i in range(m) if i not in lost][:k]
    parts = [shards[i * C:(i + 1) * C] for i in keep]
    out = ca.decoding.zfec_chunks(parts, pad, keep, k, m)
    assert out == d == O.zfec_decode_shares(parts, keep, pad, k, m)
