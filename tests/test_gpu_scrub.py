"""GPU parity: verify_slice and scrub (decoding.rs:129-212) — the per-node
bao check kernel, slice ranges, and the zfec repair path."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n", [1, 1000, 5000, 70_001])
def test_verify_slice_roundtrip(gpu, n):
    import carbonado_amd as ca
    d = _rnd(n, n)
    enc, h, info = ca.encode(b"", d, 12)
    content = O.zfec_encode(d)[0]
    # tests/codec.rs:91 — the whole stream
    assert ca.verify_slice(h, enc, 0, info.verifiable_slice_count) == content
    N = len(content) // 1024
    for index, count in [(0, 1), (1, 2), (N - 1, 1), (N // 2, N), (N + 2, 1), (3, 0)]:
        start = index * 1024
        assert ca.verify_slice(h, enc, index, count) == content[start:start + count * 1024]


def test_verify_slice_localises_corruption(gpu):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    d = _rnd(40_000, 3)
    enc, h, info = ca.encode(b"", d, 12)
    content = O.zfec_encode(d)[0]
    spc = info.chunk_slice_count
    # corrupt a byte of shard 6's first chunk (located through a 1-chunk slice)
    chunk = ca.extract_slice(enc, 6 * spc, 1)[-1024:]
    bad = bytearray(enc)
    bad[enc.index(chunk) + 17] ^= 0x80
    bad = bytes(bad)
    with pytest.raises(BaoDecodeError):
        ca.verify_slice(h, bad, 6 * spc, spc)
    for i in range(8):  # every other shard still verifies
        if i != 6:
            assert ca.verify_slice(h, bad, i * spc, spc) == content[i * spc * 1024:(i + 1) * spc * 1024]


def test_scrub_apocalypse_contract(gpu, golden_dir):
    """tests/apocalypse.rs:69-95: scrub of clean data errors; a flipped bit is
    repaired to the identical original encoding."""
    import carbonado_amd as ca
    from carbonado_amd.error import UnnecessaryScrub
    data = (golden_dir / "samples" / "contract.rgbc").read_bytes()
    enc, h, info = ca.encode(b"", data, 12)
    with pytest.raises(UnnecessaryScrub):
        ca.scrub(enc, h, info)
    bad = bytearray(enc)
    bad[6400] ^= 64
    assert ca.scrub(bytes(bad), h, info) == enc


@pytest.mark.parametrize("name", ["content.png", "code.tar"])
def test_scrub_data_shard_loss(gpu, golden_dir, name):
    """The reference's #[ignore]d apocalypse cases (tests/apocalypse.rs:22-40):
    byte 6400 falls in a DATA shard, which the reference's positional
    re-indexing cannot repair; explicit share indices can."""
    import carbonado_amd as ca
    data = (golden_dir / "samples" / name).read_bytes()
    enc, h, info = ca.encode(b"", data, 12)
    bad = bytearray(enc)
    bad[6400] ^= 64
    assert ca.scrub(bytes(bad), h, info) == enc


def test_scrub_multi_shard_and_unrecoverable(gpu):
    import carbonado_amd as ca
    from carbonado_amd.error import ZfecError
    d = _rnd(100_000, 4)
    enc, h, info = ca.encode(b"", d, 12)
    spc = info.chunk_slice_count

    def corrupt(shards):
        b = bytearray(enc)
        for i in shards:
            chunk = ca.extract_slice(enc, i * spc + 1, 1)[-1024:]
            b[enc.index(chunk) + 5] ^= 1
        return bytes(b)

    assert ca.scrub(corrupt([0, 5, 7]), h, info) == enc
    assert ca.scrub(corrupt([1, 2, 3, 4]), h, info) == enc
    with pytest.raises(ZfecError):
        ca.scrub(corrupt([0, 1, 2, 3, 4]), h, info)


@pytest.mark.parametrize("off", [0, 56])
def test_scrub_batch_matches_single(gpu, off):
    """chip_scrub_batch_dev over device-resident streams gives, object by
    object, the status and the repaired stream of the single-object scrub():
    intact, one / two / four damaged shards (the last repaired from the parity
    shards alone), five damaged shards and a damaged root node (too few
    authentic shards).  off 56: the streams 56 B into their rows (every chunk
    and node on a 64-B boundary), read and repaired there."""
    import torch
    import carbonado_amd as ca
    from carbonado_amd import device as D
    from carbonado_amd.error import CarbonadoError
    n = 50_000
    damage = [[], [2], [1, 6], [0, 1, 2, 3], [0, 1, 2, 3, 4], "root"]
    objs = [_rnd(n, 100 + i) for i in range(len(damage))]
    encs = [ca.encode(b"", d, 12) for d in objs]
    info = encs[0][2]
    spc = info.chunk_slice_count
    L = len(encs[0][0])
    bad = []
    for (enc, h, _), d, dmg in zip(encs, objs, damage):
        content = O.zfec_encode(d)[0]
        b = bytearray(enc)
        if dmg == "root":
            b[8 + 3] ^= 0x04
        else:
            for sh in dmg:
                chunk = content[sh * spc * 1024:(sh * spc + 1) * 1024]
                b[enc.index(chunk) + 100 + sh] ^= 0x21
        bad.append(bytes(b))
    count = len(bad)
    stride = (off + L + 15) // 16 * 16
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    for o in range(count):
        inp[o, off:off + L] = torch.frombuffer(bytearray(bad[o]), dtype=torch.uint8).cuda()
        hashes[o] = torch.frombuffer(bytearray(encs[o][1]), dtype=torch.uint8).cuda()
    out = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    status = D.scrub_batch(inp, L, hashes, info.padding_len, info.chunk_len, out, D.scrub_scratch(L, count),
                           offset=off)
    expect = [12, 0, 0, 0, 7, 7]
    assert list(status) == expect
    for o in range(count):
        try:
            single, st = ca.scrub(bad[o], encs[o][1], info), 0
        except CarbonadoError as e:
            single, st = None, e.status
        assert st == status[o], o
        if st == 0:
            assert single == encs[o][0]
            assert bytes(out[o, off:off + L].cpu().numpy()) == encs[o][0]
