"""Seeded randomized parity: the device batch paths against the C oracle over
sizes drawn around the boundaries the kernels branch on (1 KiB chunks, 4 KiB
zfec tiles, 8 KiB column groups, 64 KiB content-mode blocks, 32 KiB level-12
full blocks), random batch counts, row strides and output line phases, and
random zfec shapes with random erasure sets, and every format level over
compressible data (the host Snappy stage's copy and literal paths).  Every case is bit-exact or the
test fails; the seeds are fixed, so a failure reproduces."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

BOUNDARIES = [1024, 4096, 8192, 32768, 65536, 131072, 1 << 20]


def draw_size(rng) -> int:
    base = int(rng.choice(BOUNDARIES)) * int(rng.integers(1, 4))
    return max(1, base + int(rng.integers(-70, 71)))


@pytest.mark.parametrize("case", range(40))
def test_encode_decode_batch_dev_random(gpu, case):
    """chip_encode_batch_dev then chip_decode_batch_dev at a random device-only
    level: every object's encoding equals the oracle's encode(), every object
    decodes back (status 0), nothing is written past an encoding."""
    import torch
    from carbonado_amd import device
    rng = np.random.default_rng(0xF022 + case)
    level = int(rng.choice([4, 8, 12]))
    n = draw_size(rng)
    count = int(rng.integers(1, 5))
    stride = (n + int(rng.integers(0, 64)) + 15) // 16 * 16
    host = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    cap = device._lib.lib().chip_encode_max_len(n)
    ostride = (cap + 15) // 16 * 16 + 16 * int(rng.integers(0, 8))
    # level 12 streams of more than 512 chunks at a random 8-B phase in their rows
    off = 8 * int(rng.integers(0, 32)) if level == 12 and n > 300 * 1024 else 0
    out = torch.full((count, ostride + (256 if off else 0)), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    olen, info = device.encode_batch(level, inp, n, out, hashes, device.encode_scratch(level, n, count),
                                     out_offset=off)
    torch.cuda.synchronize()
    got, gh = out.cpu().numpy(), hashes.cpu().numpy()
    for o in range(count):
        enc, h, oinfo = O.encode(host[o, :n].tobytes(), level)
        assert olen == len(enc), (level, n)
        assert got[o, off:off + olen].tobytes() == enc, (level, n, o, off)
        assert (got[o, :off] == 0xA5).all() and (got[o, off + olen:] == 0xA5).all(), (level, n, o, off)
        if level & 4:
            assert gh[o].tobytes() == h, (level, n, o)
    dec = torch.full((count, stride), 0x5A, dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    dlen = device.decode_batch(level, out, olen, hashes, info.padding_len, dec, status,
                               device.decode_scratch(level, olen, count), in_offset=off)
    torch.cuda.synchronize()
    assert dlen == n and status.cpu().tolist() == [0] * count
    assert np.array_equal(dec.cpu().numpy()[:, :n], host[:, :n])


@pytest.mark.parametrize("case", range(24))
def test_bao_batch_random_line_phase(gpu, case):
    """bao encode of a random batch (content mode from 64 KiB, K3 below) with
    an output stride of 8 mod 16, so object bases take varying 8-B phases of
    a 128-B line."""
    import torch
    from carbonado_amd import device
    rng = np.random.default_rng(0xBA0 + case)
    n = draw_size(rng)
    count = int(rng.integers(2, 6))
    blen = O.lib().orc_bao_encoded_len(n)
    stride = (blen + 15) // 16 * 16 + 8 + 16 * int(rng.integers(0, 8))
    istride = (n + 15) // 16 * 16
    host = rng.integers(0, 256, (count, istride), dtype=np.uint8)
    out = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    device.bao_encode_batch(torch.from_numpy(host).cuda(), n, out, hashes, device.bao_scratch(n, count))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for o in range(count):
        oe, oh = O.bao_encode(host[o, :n].tobytes())
        assert hashes[o].cpu().numpy().tobytes() == oh, (n, o)
        assert got[o, :blen].tobytes() == oe, (n, o)
        assert (got[o, blen:] == 0xA5).all(), (n, o)


@pytest.mark.parametrize("case", range(32))
def test_zfec_random_shape_and_erasures(gpu, case):
    """zfec k-of-m encode of a random size and shape (k up to 20, m up to
    k + 12), then decode from a random k-subset of the shares given with
    their true indices; the shards equal the oracle's."""
    from carbonado_amd import decoding, encoding
    rng = np.random.default_rng(0x2FEC + case)
    k = int(rng.integers(1, 21))
    m = k + int(rng.integers(1, 13))
    n = draw_size(rng) // 4 + 1
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    z, pad, C = encoding.zfec(d, k, m)
    oz, opad, oC = O.zfec_encode(d, k, m)
    assert (pad, C) == (opad, oC) and z == oz, (k, m, n)
    keep = sorted(rng.choice(m, size=k, replace=False).tolist())
    shares = [z[i * C:(i + 1) * C] for i in keep]
    assert decoding.zfec_chunks(shares, pad, indices=keep, k=k, m=m) == d, (k, m, n, keep)


def compressible(rng, n: int) -> bytes:
    """Bytes snappy compresses in every way it can: runs, back-references at
    random distances and lengths (short and long copies, overlapping ones),
    and literal stretches."""
    out = bytearray()
    while len(out) < n:
        kind = int(rng.integers(0, 4))
        if kind == 0 or len(out) < 8:
            out += rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
        elif kind == 1:
            out += bytes([int(rng.integers(0, 256))]) * int(rng.integers(4, 3000))
        else:
            dist = int(rng.integers(1, min(len(out), 70_000) + 1))
            ln = int(rng.integers(4, 300))
            start = len(out) - dist
            for i in range(ln):
                out.append(out[start + i])
    return bytes(out[:n])


@pytest.mark.parametrize("case", range(32))
def test_every_level_compressible_random(gpu, case):
    """encode() at a random level of compressible data with the ECIES
    randomness injected == the C oracle's full pipeline; decode() inverts it."""
    import carbonado_amd as ca
    from oracle import host_oracle as H
    rng = np.random.default_rng(0xC0DE + case)
    level = int(rng.integers(0, 16))
    n = int(rng.choice([int(rng.integers(0, 5000)), draw_size(rng), int(rng.integers(300_000, 1_500_000))]))
    d = compressible(rng, n)
    sk = H.sha256(b"fuzz receiver %d" % case)
    pub = H.public_key(sk)
    eph = H.sha256(b"fuzz eph %d" % case)
    nonce = H.sha256(b"fuzz nonce %d" % case)[:16]
    enc, h, info = ca.encode(pub, d, level, ephemeral_sk=eph, nonce=nonce)
    oenc, oh, oinfo = O.c_encode_full(d, level, pub, eph, nonce)
    assert enc == oenc and h == oh, (level, n)
    assert info.padding_len == oinfo["padding_len"], (level, n)
    assert ca.decode(sk, h, enc, info.padding_len, level) == d, (level, n)


def chunk_off(i: int, N: int) -> int:
    """Stream offset of chunk i of an N-chunk bao stream: 8 + 1024 i + 64 (P(i) + c(i))."""
    def clog2(x):
        return 0 if x <= 1 else (x - 1).bit_length()
    cl = clog2(N - i)
    c = cl if i == 0 else min((i & -i).bit_length() - 1, cl)
    total, cnt, L = 0, N, 1
    while cnt > 1:
        total += min((i + (1 << L) - 1) >> L, cnt // 2)
        cnt = (cnt + 1) // 2
        L += 1
    return 8 + 1024 * i + 64 * (total + c)


@pytest.mark.parametrize("case", range(12))
def test_scrub_random_shard_corruption(gpu, case):
    """scrub() (decoding.rs:159-212) of a level-12 stream with content bytes
    flipped inside a random set of shards: up to m - k = 4 damaged shards are
    repaired bit-exactly (true share indices), 5 or more fail with a zfec
    error, an intact stream is UnnecessaryScrub."""
    import carbonado_amd as ca
    from carbonado_amd.error import UnnecessaryScrub, ZfecError
    rng = np.random.default_rng(0x5C2B + case)
    n = draw_size(rng) // 2 + 1
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, h, info = ca.encode(b"", d, 12)
    cols = info.chunk_len // 1024
    N = 8 * cols
    with pytest.raises(UnnecessaryScrub):
        ca.scrub(enc, h, info)
    nbad = int(rng.integers(1, 7))
    shards = sorted(rng.choice(8, size=nbad, replace=False).tolist())
    bad = bytearray(enc)
    for s in shards:  # distinct content bytes of the shard, so no flip undoes another
        for pos in rng.choice(cols * 1024, size=int(rng.integers(1, 4)), replace=False).tolist():
            i = s * cols + pos // 1024
            bad[chunk_off(i, N) + pos % 1024] ^= 1 << int(rng.integers(0, 8))
    if nbad <= 4:
        assert ca.scrub(bytes(bad), h, info) == enc, (n, shards)
    else:
        with pytest.raises(ZfecError):
            ca.scrub(bytes(bad), h, info)


@pytest.mark.parametrize("case", range(24))
def test_decode_malformed_inputs_random(gpu, case):
    """decode() of damaged encodings: a CarbonadoError, never a crash, and
    never a wrong answer where the format can tell (a flipped byte at a level
    with Bao or Ecies, a truncated encoding, random bytes of a random
    length)."""
    import carbonado_amd as ca
    from carbonado_amd.error import CarbonadoError
    from oracle import host_oracle as H
    rng = np.random.default_rng(0xDEAD + case)
    level = int(rng.integers(0, 16))
    n = int(rng.choice([int(rng.integers(1, 3000)), draw_size(rng) // 4 + 1]))
    d = compressible(rng, n) if case % 2 else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    sk = H.sha256(b"malformed %d" % case)
    enc, h, info = ca.encode(H.public_key(sk), d, level)
    assert ca.decode(sk, h, enc, info.padding_len, level) == d
    # Bao verifies every byte of the encoding; the AES-GCM tag every byte that
    # decryption reads (without Bao, zfec decode reads the data shards only, so
    # a flip in a parity shard or the padding is harmless and goes unnoticed,
    # as in the reference); levels 0, 2, 8, 10 have no integrity check at all
    detects = bool(level & 4) or bool(level & 1)

    def outcome(buf):
        try:
            return ca.decode(sk, h, buf, info.padding_len, level)
        except CarbonadoError:
            return None
    flipped = bytearray(enc)
    flipped[int(rng.integers(0, len(enc)))] ^= 1 << int(rng.integers(0, 8))
    got = outcome(bytes(flipped))
    if level & 4:
        assert got is None, (level, n)
    elif level & 1:
        assert got is None or got == d, (level, n)
    if len(enc) > 1:
        got = outcome(enc[:int(rng.integers(0, len(enc)))])
        if detects:
            assert got is None, (level, n)
    junk = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
    try:
        out = ca.decode(sk, h, junk, info.padding_len, level)
        assert not detects, "random bytes decoded at a level that verifies its input"
        assert isinstance(out, bytes)
    except CarbonadoError:
        pass
