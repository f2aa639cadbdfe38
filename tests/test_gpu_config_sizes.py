"""GPU parity at BASELINE.json's own object size (16 MiB), one object per
config, against the C oracle:

* cfg4: the full level-15 encode() of a 16 MiB random object with the ECIES
  randomness injected (N = 32776 chunks, padding 1941, C = 4,195,328 — not a
  multiple of K1's 4 KiB tile), bit-exact against host_oracle.c's
  orc_encode_full, and decoded back;
* cfg5 shape: zfec 8-of-16 encode of 16 MiB, then decode with 8 shards
  dropped (data and parity mixed);
* cfg3: every one of the 28 two-erasure patterns of 4-of-8 on one 16 MiB
  object, decoded on the device and compared with the input;
* the level-12 device pipeline at 16 MiB (the fused zfec + bao kernel with
  tree levels 1-3 in the wave, its full-block path), streams and hashes
  bit-exact for several objects and stream placements.
"""
import itertools

import numpy as np
import pytest

from oracle import host_oracle as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 16 << 20
SK = H.sha256(b"config-size receiver")
EPH = H.sha256(b"config-size ephemeral")
NONCE = H.sha256(b"config-size nonce")[:16]


@pytest.fixture(scope="module")
def obj16():
    return np.random.default_rng(16).integers(0, 256, N, dtype=np.uint8).tobytes()


def test_cfg4_level15_16mib_bit_exact(gpu, obj16):
    import carbonado_amd as ca
    pub = O.c_public_key(SK)
    enc, h, info = ca.encode(pub, obj16, 15, ephemeral_sk=EPH, nonce=NONCE)
    oenc, oh, oinfo = O.c_encode_full(obj16, 15, pub, EPH, NONCE)
    assert info.padding_len == 1941 and info.chunk_len == 4_195_328
    assert info.bytes_ecc == 8 * 4_195_328 and info.verifiable_slice_count == 32776
    assert len(enc) == len(oenc) == info.bytes_verifiable == 35_660_232
    assert h == oh
    assert O.blake3(enc) == O.blake3(oenc)
    assert enc == oenc
    assert ca.decode(SK, h, enc, info.padding_len, 15) == obj16


def test_cfg5_8of16_16mib_encode_and_decode_8_lost(gpu, obj16):
    import torch
    from carbonado_amd import device
    inp = torch.from_numpy(np.frombuffer(obj16, np.uint8).copy()).cuda().reshape(1, N)
    C = N // 8
    enc = torch.zeros((1, 16 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, enc, 8, 16)
    torch.cuda.synchronize()
    ref, pad, oC = O.zfec_encode(obj16, 8, 16)
    assert pad == 0 and oC == C
    got = enc[0].cpu().numpy().tobytes()
    assert got == ref
    lost = {1, 2, 5, 7, 8, 11, 12, 15}  # 4 data + 4 parity shards
    keep = [i for i in range(16) if i not in lost]
    out = torch.zeros((1, N), dtype=torch.uint8, device="cuda")
    device.zfec_decode_batch(enc, C, keep, out, 8, 16)
    torch.cuda.synchronize()
    assert out[0].cpu().numpy().tobytes() == obj16
    # the C oracle's share-matrix decode agrees
    shares = [ref[i * C:(i + 1) * C] for i in keep]
    assert O.zfec_decode_shares(shares, keep, 0, 8, 16) == obj16


def test_cfg3_all_28_erasure_pairs_16mib(gpu, obj16):
    import torch
    from carbonado_amd import device
    inp = torch.from_numpy(np.frombuffer(obj16, np.uint8).copy()).cuda().reshape(1, N)
    C = N // 4
    enc = torch.zeros((1, 8 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, enc, 4, 8)
    torch.cuda.synchronize()
    assert enc[0].cpu().numpy().tobytes() == O.zfec_encode(obj16)[0]
    pairs = list(itertools.combinations(range(8), 2))
    assert len(pairs) == 28
    out = torch.zeros((len(pairs), N), dtype=torch.uint8, device="cuda")
    for i, lost in enumerate(pairs):
        keep = [s for s in range(8) if s not in lost]
        device.zfec_decode_batch(enc, C, keep, out[i:i + 1], 4, 8)
    torch.cuda.synchronize()
    for i, lost in enumerate(pairs):
        assert torch.equal(out[i], inp[0]), lost


@pytest.mark.parametrize("shift", [0, 112])
def test_level12_16mib_fused_full_path(gpu, obj16, shift):
    """encode_batch at Zfec|Bao on 3 x 16 MiB objects (C = 4 MiB: 4096 chunk
    columns, no zfec padding: the fused kernel's FULL path) against the
    oracle's encode(); shift 112 moves every chunk to another phase of the
    128-B memory lines (the line stores' head and tail pieces)."""
    import torch
    from carbonado_amd import device
    objs = [obj16, bytes(reversed(obj16)), np.random.default_rng(12).integers(0, 256, N, np.uint8).tobytes()]
    oenc = [O.encode(o, 12) for o in objs]
    blen = len(oenc[0][0])
    stride = (blen + shift + 255) // 256 * 256
    inp = torch.from_numpy(np.frombuffer(b"".join(objs), np.uint8).copy()).cuda().reshape(3, N)
    raw = torch.full((3 * stride + 256,), 0xA5, dtype=torch.uint8, device="cuda")
    out = raw[shift:shift + 3 * stride].view(3, stride)
    hashes = torch.zeros((3, 32), dtype=torch.uint8, device="cuda")
    olen, info = device.encode_batch(12, inp, N, out, hashes, device.encode_scratch(12, N, 3))
    torch.cuda.synchronize()
    assert olen == blen and info.padding_len == 0
    got, gh = out.cpu().numpy(), hashes.cpu().numpy()
    for o, (enc, h, _) in enumerate(oenc):
        assert got[o, :blen].tobytes() == enc, o
        assert gh[o].tobytes() == h
        assert (got[o, blen:] == 0xA5).all()


def test_zfec_linearity_16mib_batch(gpu):
    """A size-independent property at the config size: zfec encode is linear
    over GF(2^8), so the shards of A xor B are the xor of the shards of A and
    of B (8 objects of 16 MiB, 4-of-8 and 8-of-16), and the data shards are
    the input itself (systematic code)."""
    import torch
    from carbonado_amd import device
    g = torch.Generator(device="cuda").manual_seed(1616)
    a = torch.randint(0, 256, (8, N), dtype=torch.uint8, device="cuda", generator=g)
    b = torch.randint(0, 256, (8, N), dtype=torch.uint8, device="cuda", generator=g)
    for k, m in ((4, 8), (8, 16)):
        C = N // k
        outs = []
        for x in (a, b, a ^ b):
            o = torch.empty((8, m * C), dtype=torch.uint8, device="cuda")
            device.zfec_encode_batch(x, N, o, k, m)
            outs.append(o)
        torch.cuda.synchronize()
        assert torch.equal(outs[2], outs[0] ^ outs[1])
        assert torch.equal(outs[0][:, :N], a)


def test_level15_shape_batch_level12_bit_exact(gpu):
    """The zfec + bao device batch at the shard length level 15 produces for a
    16 MiB object (16,779,371 B after snap + ECIES: 4097-chunk shards, 8 does
    not divide the column count, padding 1941): the fused kernel's general
    path, then tree levels 1-3 in one pass (bao_levels123_kernel) and the
    parent kernels from level 4.  Every stream and hash against the oracle."""
    import torch
    from carbonado_amd import _lib, device
    L = _lib.lib()
    n, count = 16_779_371, 3
    rng = np.random.default_rng(1515)
    host = rng.integers(0, 256, (count, n), dtype=np.uint8)
    row = (n + 15) // 16 * 16
    inp = torch.zeros((count, row), dtype=torch.uint8)
    inp[:, :n] = torch.from_numpy(host)
    inp = inp.cuda()
    zlen = 8 * 4_195_328
    blen = L.chip_bao_encoded_len(zlen)
    out = torch.zeros((count, (blen + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    scratch = device.encode_scratch(12, n, count)
    _, info = device.encode_batch(12, inp, n, out, hashes, scratch)
    torch.cuda.synchronize()
    assert info.padding_len == 1941 and info.chunk_len == 4_195_328
    for o in range(count):
        enc, h, _ = O.encode(host[o].tobytes(), 12)
        assert len(enc) == blen
        assert out[o, :blen].cpu().numpy().tobytes() == enc, o
        assert hashes[o].cpu().numpy().tobytes() == h, o


@pytest.mark.parametrize("level", [12, 4])
@pytest.mark.parametrize("n", [N, 16_779_371])
def test_fused_64bit_address_forms_match(gpu, monkeypatch, level, n):
    """The fused kernels address every object through 32-bit lane offsets from
    its base when the shard length is < 256 MiB (all BASELINE sizes), and
    through 64-bit addresses above that.  CHIP_K13_O32=0 forces the 64-bit
    forms at this size: both must give the oracle's streams and hashes (level
    12: zfec + bao, FULL path at 16 MiB, general path at the level-15 shard
    length; level 4: bao of the content, content mode + tail kernel)."""
    import torch
    from carbonado_amd import device
    rng = np.random.default_rng(n + level)
    count = 2
    host = rng.integers(0, 256, (count, n), dtype=np.uint8)
    row = (n + 15) // 16 * 16
    inp = torch.zeros((count, row), dtype=torch.uint8)
    inp[:, :n] = torch.from_numpy(host)
    inp = inp.cuda()
    outs = []
    for o32 in ("1", "0"):
        monkeypatch.setenv("CHIP_K13_O32", o32)
        scratch = device.encode_scratch(level, n, count)
        oenc = O.encode(host[0].tobytes(), level)
        blen = len(oenc[0])
        out = torch.zeros((count, (blen + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
        hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
        olen, _ = device.encode_batch(level, inp, n, out, hashes, scratch)
        torch.cuda.synchronize()
        assert olen == blen
        outs.append((out.cpu(), hashes.cpu()))
        assert out[0, :blen].cpu().numpy().tobytes() == oenc[0]
        assert hashes[0].cpu().numpy().tobytes() == oenc[1]
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
