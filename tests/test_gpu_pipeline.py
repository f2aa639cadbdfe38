"""GPU parity: encode()/decode() glue for the Bao|Zfec levels on the
reference's own samples (tests/codec.rs and tests/apocalypse.rs restated
for the deterministic levels; ECIES/Snappy are host stages out of scope)."""
import json

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SAMPLES = ["contract.rgbc", "content.png", "code.tar"]


@pytest.fixture(scope="module")
def golden(golden_dir):
    return json.loads((golden_dir / "golden.json").read_text())


@pytest.mark.parametrize("name", SAMPLES)
@pytest.mark.parametrize("level", [0, 4, 8, 12])
def test_codec_samples(gpu, golden, golden_dir, name, level):
    import carbonado_amd as ca
    data = (golden_dir / "samples" / name).read_bytes()
    enc, h, info = ca.encode(b"", data, level)
    if level:
        g = golden["samples"][name][f"level{level}"]
        assert h.hex() == g["hash"]
        assert len(enc) == g["output_len"]
        assert O.blake3(enc).hex() == g["output_blake3"]
        for k, v in g["info"].items():
            assert getattr(info, k) == pytest.approx(v, rel=1e-6), k
    else:
        assert enc == data and h == b"\0" * 32
    # tests/codec.rs:84-88
    if level & 4:
        assert len(enc) == info.bytes_verifiable
    # tests/codec.rs:94-101
    assert ca.decode(b"", h, enc, info.padding_len, level) == data


def test_apocalypse_bitflip_detected_and_recovered(gpu, golden_dir):
    """tests/apocalypse.rs:69-95 at level 12: a flipped bit fails bao
    verification; the surviving shards (explicit indices) restore the data."""
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError
    data = (golden_dir / "samples" / "contract.rgbc").read_bytes()
    enc, h, info = ca.encode(b"", data, 12)
    bad = bytearray(enc)
    bad[6400] ^= 64
    with pytest.raises(BaoDecodeError):
        ca.decode(b"", h, bytes(bad), info.padding_len, 12)
    # shard 5 (parity) holds byte 6400 for this sample: drop it, decode from the rest
    z, pad, C = ca.encoding.zfec(data)
    keep = [i for i in range(8) if i != 5]
    shards = [z[i * C:(i + 1) * C] for i in keep]
    assert ca.decoding.zfec_chunks(shards, pad, indices=keep) == data
    # re-encoding reproduces the original stream bit for bit (scrub's check)
    re_enc, re_h = ca.encoding.bao(ca.encoding.zfec(ca.decoding.zfec_chunks(shards, pad, indices=keep))[0])
    assert re_enc == enc and re_h == h


@pytest.mark.parametrize("n", [0, 1, 4096, 10_000, (1 << 20) + 1])
def test_levels_random(gpu, n):
    import carbonado_amd as ca
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    for level in (4, 8, 12):
        enc, h, info = ca.encode(b"", d, level)
        oenc, oh, oinfo = O.encode(d, level)
        assert enc == oenc and h == oh
        assert ca.decode(b"", h, enc, info.padding_len, level) == d


@pytest.mark.parametrize("level", [4, 8, 12])
@pytest.mark.parametrize("pinned", [False, True])
def test_encode_host_batch(gpu, level, pinned):
    """chip_encode_host_batch (pipelined host->HBM->host) == encode() per object."""
    import torch
    from carbonado_amd import device
    n, count = 70_001, 7
    rng = np.random.default_rng(level)
    inp = torch.from_numpy(rng.integers(0, 256, (count, n + 9), dtype=np.uint8))  # ragged stride
    if pinned:
        inp = inp.pin_memory()
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.zeros((count, cap + 5), dtype=torch.uint8)
    hashes = torch.zeros((count, 32), dtype=torch.uint8)
    if pinned:
        out, hashes = out.pin_memory(), hashes.pin_memory()
    olen, info = device.encode_host_batch(level, inp, n, out, hashes, nslots=2, slice_bytes=3 * n)
    for o in range(count):
        enc, h, oinfo = O.encode(inp[o, :n].numpy().tobytes(), level)
        assert olen == len(enc)
        assert out[o, :olen].numpy().tobytes() == enc, o
        assert hashes[o].numpy().tobytes() == (h if level & 4 else b"\0" * 32)
    assert info.output_len == olen and info.padding_len == oinfo["padding_len"]


def test_bao_decode_batch_header_mismatch(gpu):
    import torch
    from carbonado_amd import device
    n = 5000
    d = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, h = O.bao_encode(d)
    t = torch.from_numpy(np.frombuffer(enc + b"\0" * 8, np.uint8).copy()).cuda().reshape(1, -1)
    t[0, 0] ^= 1  # header says n ^ 1
    hashes = torch.from_numpy(np.frombuffer(h, np.uint8).copy()).cuda().reshape(1, 32)
    out = torch.empty((1, n), dtype=torch.uint8, device="cuda")
    status = torch.empty(1, dtype=torch.int32, device="cuda")
    device.bao_decode_batch(t, n, hashes, out, status, device.bao_scratch(n, 1))
    torch.cuda.synchronize()
    assert int(status[0]) == 5
