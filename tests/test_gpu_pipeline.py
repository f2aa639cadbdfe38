"""GPU parity: encode()/decode() glue on the reference's own samples
(tests/codec.rs and tests/apocalypse.rs restated) for every format level:
Bao|Zfec on the device, Snappy/Ecies as host stages with the ECIES
randomness injected so the output is bit-comparable with the oracle."""
import json

import numpy as np
import pytest

from oracle import host_oracle as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SK = H.sha256(b"pipeline receiver")
PUB = H.public_key(SK)
EPH = H.sha256(b"pipeline ephemeral")
NONCE = H.sha256(b"pipeline nonce")[:16]

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


@pytest.mark.parametrize("level", [4, 5, 6])
def test_encode_host_batch_bao_only_large(gpu, level):
    """Bao without Zfec from host memory, streams of more than 512 chunks: the
    slot rows hold them 56 B in (K3 / the content mode at that phase) and the
    copy back reads them from there; == encode() per object."""
    import torch
    from carbonado_amd import device
    n, count = (600 << 10) + 13, 3
    rng = np.random.default_rng(level + 40)
    inp = torch.from_numpy(rng.integers(0, 256, (count, n), dtype=np.uint8)).pin_memory()
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.full((count, cap), 0xA5, dtype=torch.uint8).pin_memory()
    hashes = torch.zeros((count, 32), dtype=torch.uint8).pin_memory()
    eph = np.stack([np.frombuffer(H.sha256(b"bo%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"bn%d" % o)[:16], np.uint8) for o in range(count)])
    olen, _ = device.encode_host_batch(level, inp, n, out, hashes, nslots=2, slice_bytes=2 * n, pubkey=PUB,
                                       ephemeral_sk=eph, nonce=nonce, host_threads=3)
    for o in range(count):
        enc, h, _ = O.encode_full(inp[o].numpy().tobytes(), level, PUB, eph[o].tobytes(), nonce[o].tobytes())
        assert out[o, :olen[o]].numpy().tobytes() == enc and hashes[o].numpy().tobytes() == h, o


@pytest.mark.parametrize("level", [4, 8, 12, 15])
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
    eph = np.stack([np.frombuffer(H.sha256(b"eph%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"nonce%d" % o)[:16], np.uint8) for o in range(count)])
    olen, info = device.encode_host_batch(level, inp, n, out, hashes, nslots=2, slice_bytes=3 * n, pubkey=PUB,
                                          ephemeral_sk=eph, nonce=nonce, host_threads=3)
    for o in range(count):
        enc, h, oinfo = O.encode_full(inp[o, :n].numpy().tobytes(), level, PUB, eph[o].tobytes(),
                                      nonce[o].tobytes())
        assert olen[o] == len(enc)
        assert out[o, :olen[o]].numpy().tobytes() == enc, o
        assert hashes[o].numpy().tobytes() == (h if level & 4 else b"\0" * 32)
        assert info[o].output_len == olen[o] and info[o].padding_len == oinfo["padding_len"]
        assert info[o].bytes_encrypted == oinfo["bytes_encrypted"]
        assert info[o].bytes_compressed == oinfo["bytes_compressed"]


def test_encode_host_batch_ragged_host_stage_sizes(gpu):
    """Compressible objects give different snap sizes per object: the batch
    falls back to per-object device launches inside a slice."""
    import torch
    from carbonado_amd import device
    n, count = 50_000, 5
    rng = np.random.default_rng(77)
    rows = [rng.integers(0, 256, n, dtype=np.uint8), np.zeros(n, np.uint8),
            rng.integers(0, 3, n, dtype=np.uint8), np.frombuffer((b"carbonado " * n)[:n], np.uint8),
            rng.integers(0, 256, n, dtype=np.uint8)]
    inp = torch.from_numpy(np.stack(rows))
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.zeros((count, cap), dtype=torch.uint8)
    hashes = torch.zeros((count, 32), dtype=torch.uint8)
    eph = np.stack([np.frombuffer(H.sha256(b"r%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"q%d" % o)[:16], np.uint8) for o in range(count)])
    for level in (14, 15):
        olen, info = device.encode_host_batch(level, inp, n, out, hashes, nslots=2, slice_bytes=2 * n,
                                              pubkey=PUB, ephemeral_sk=eph, nonce=nonce)
        assert len(set(olen)) > 1
        for o in range(count):
            enc, h, oinfo = O.encode_full(rows[o].tobytes(), level, PUB, eph[o].tobytes(), nonce[o].tobytes())
            assert out[o, :olen[o]].numpy().tobytes() == enc and hashes[o].numpy().tobytes() == h, (level, o)


@pytest.mark.parametrize("n", [(1 << 20) + 5, 3 << 20])
@pytest.mark.parametrize("level", [12, 15])
@pytest.mark.parametrize("soff", ["0", "120"])
def test_encode_host_batch_stream_offset(gpu, level, n, soff, monkeypatch):
    """The slot rows hold K13's streams CHIP_STREAM_OFFSET bytes in (default
    56: every chunk and node on a 64-B boundary, covered by the split
    copy-back test); at the row start and at another 8-B phase the split
    copy-back, the node gather and the whole-stream copy give the same bytes."""
    monkeypatch.setenv("CHIP_STREAM_OFFSET", soff)
    test_encode_host_batch_split_copy_back(gpu, level, n)


@pytest.mark.parametrize("n", [1, 1000, 4096, 70_001, (1 << 20) + 5, 3 << 20])
@pytest.mark.parametrize("level", [12, 13, 14, 15])
def test_encode_host_batch_split_copy_back(gpu, level, n):
    """Zfec|Bao from host memory: the host writes each stream's header and
    data-shard chunks itself, the device gathers the parent nodes between them
    and the tail crosses PCIe (api_encode.cpp SplitGeo).  Output pre-filled with
    0xA5 so a byte nobody wrote shows; nine objects over two slots of two
    objects each, so slots are reused and nodes scattered while the next slice
    stages; count 1 separately (pitch = the stream length)."""
    import torch
    from carbonado_amd import device
    count = 9
    rng = np.random.default_rng(n + level)
    inp = torch.from_numpy(rng.integers(0, 256, (count, n + 3), dtype=np.uint8)).pin_memory()
    cap = device._lib.lib().chip_encode_max_len(n)
    eph = np.stack([np.frombuffer(H.sha256(b"s%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"t%d" % o)[:16], np.uint8) for o in range(count)])
    for cnt in (count, 1):
        out = torch.full((cnt, cap + 8), 0xA5, dtype=torch.uint8).pin_memory()
        hashes = torch.zeros((cnt, 32), dtype=torch.uint8).pin_memory()
        olen, _ = device.encode_host_batch(level, inp[:cnt], n, out, hashes, nslots=2, slice_bytes=2 * n + 2,
                                           pubkey=PUB, ephemeral_sk=eph[:cnt], nonce=nonce[:cnt], host_threads=3)
        for o in range(cnt):
            enc, h, _ = O.encode_full(inp[o, :n].numpy().tobytes(), level, PUB, eph[o].tobytes(),
                                      nonce[o].tobytes())
            assert olen[o] == len(enc)
            assert out[o, :olen[o]].numpy().tobytes() == enc, (cnt, o)
            assert hashes[o].numpy().tobytes() == h
            assert (out[o, olen[o]:].numpy() == 0xA5).all()  # nothing past the stream


@pytest.mark.parametrize("level", [14, 15])
@pytest.mark.parametrize("kind", ["ragged", "uniform_compressible"])
def test_encode_host_batch_direct_fallbacks(gpu, kind, level):
    """Pinned output at (Ecies|)Snappy|Zfec|Bao: the host stage writes straight
    into the chunk slots laid out for the incompressible size.  Objects that
    compress get another geometry: their output is read back from the slots
    and placed again (ragged slices: per-object launches; a uniform slice of
    equally compressible objects: the staged split path).  Every object equals
    the oracle's, nothing is written past a stream."""
    import torch
    from carbonado_amd import device
    n = 150_000
    rng = np.random.default_rng(31)
    if kind == "ragged":
        rows = [rng.integers(0, 256, n, dtype=np.uint8), np.zeros(n, np.uint8),
                rng.integers(0, 256, n, dtype=np.uint8), np.frombuffer((b"carbonado " * n)[:n], np.uint8),
                rng.integers(0, 256, n, dtype=np.uint8), rng.integers(0, 3, n, dtype=np.uint8)]
    else:
        rows = [np.frombuffer((b"abcdefgh" * n)[:n], np.uint8) for _ in range(6)]
    count = len(rows)
    inp = torch.from_numpy(np.stack(rows)).pin_memory()
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.full((count, cap + 8), 0xA5, dtype=torch.uint8).pin_memory()
    hashes = torch.zeros((count, 32), dtype=torch.uint8).pin_memory()
    eph = np.stack([np.frombuffer(H.sha256(b"f%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"g%d" % o)[:16], np.uint8) for o in range(count)])
    olen, _ = device.encode_host_batch(level, inp, n, out, hashes, nslots=2, slice_bytes=2 * n, pubkey=PUB,
                                       ephemeral_sk=eph, nonce=nonce, host_threads=2)
    for o in range(count):
        enc, h, _ = O.encode_full(rows[o].tobytes(), level, PUB, eph[o].tobytes(), nonce[o].tobytes())
        assert out[o, :olen[o]].numpy().tobytes() == enc and hashes[o].numpy().tobytes() == h, o
        assert (out[o, olen[o]:].numpy() == 0xA5).all(), o


@pytest.mark.parametrize("name", SAMPLES)
@pytest.mark.parametrize("level", [1, 2, 3, 14, 15])
def test_codec_samples_host_levels(gpu, golden, golden_dir, name, level):
    """tests/codec.rs:84-101 at the host-stage levels, against golden.json
    (ECIES material injected as make_golden.py does)."""
    import carbonado_amd as ca
    m = golden["ecies_material"]
    sk, eph, nonce = (bytes.fromhex(m[k]) for k in ("secret_key", "ephemeral_sk", "nonce"))
    data = (golden_dir / "samples" / name).read_bytes()
    enc, h, info = ca.encode(bytes.fromhex(m["public_key"]), data, level, ephemeral_sk=eph, nonce=nonce)
    g = golden["samples"][name][f"level{level}"]
    assert h.hex() == g["hash"] and len(enc) == g["output_len"]
    assert O.blake3(enc).hex() == g["output_blake3"]
    for k, v in g["info"].items():
        assert getattr(info, k) == pytest.approx(v, rel=1e-6), k
    if level & 4:
        assert len(enc) == info.bytes_verifiable
        # tests/codec.rs:90-91 verify_slice over the whole stream
        assert ca.verify_slice(h, enc, 0, info.verifiable_slice_count) is not None
    assert ca.decode(sk, h, enc, info.padding_len, level) == data


@pytest.mark.parametrize("n", [0, 1, 1000, 70_000, (1 << 20) + 3])
def test_every_level_random_keys(gpu, n):
    """Reference-style use: fresh ephemeral keys (no injection), every level
    round-trips and the device stages match the oracle on the same envelope."""
    import carbonado_amd as ca
    rng = np.random.default_rng(n + 1)
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes() if n % 2 else (b"abcdefgh" * (n // 8 + 1))[:n]
    for level in range(16):
        enc, h, info = ca.encode(PUB, d, level)
        assert ca.decode(SK, h, enc, info.padding_len, level) == d, level
        if level & 1:  # the envelope is random: re-derive the expected stream from it
            envelope = O.decode(h, enc, info.padding_len, level & 12) if level & 12 else enc
            assert H.ecies_decrypt(SK, envelope) == (H.snap_compress(d) if level & 2 else d)
        else:
            oenc, oh, _ = O.encode_full(d, level)
            assert enc == oenc and h == oh, level


def test_decode_host_stage_errors(gpu):
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError, EciesError
    d = b"secret payload " * 500
    enc, h, info = ca.encode(PUB, d, 15)
    with pytest.raises(EciesError):
        ca.decode(H.sha256(b"wrong key"), h, enc, info.padding_len, 15)
    bad = bytearray(enc)
    bad[len(bad) // 2] ^= 1
    with pytest.raises(BaoDecodeError):
        ca.decode(SK, h, bytes(bad), info.padding_len, 15)
    # without bao the tampered envelope is caught by the AES-GCM tag
    enc11, h11, info11 = ca.encode(PUB, d, 11)
    bad = bytearray(enc11)
    bad[200] ^= 1
    with pytest.raises(EciesError):
        ca.decode(SK, h11, bytes(bad), info11.padding_len, 11)


def test_decode_grows_output_for_compressible_data(gpu):
    """Snappy output size is known only after decompression: decode() retries
    with the size the library reports (CHIP_ERR_BUFFER_TOO_SMALL)."""
    import carbonado_amd as ca
    d = bytes(3 << 20)  # compresses ~20x
    enc, h, info = ca.encode(PUB, d, 14)
    assert len(enc) < len(d) // 4
    assert ca.decode(b"", h, enc, info.padding_len, 14) == d


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


@pytest.mark.parametrize("level", [4, 8, 12, 14, 15])
def test_decode_host_batch_roundtrip(gpu, level):
    """chip_decode_host_batch (host -> HBM -> host decode()) inverts the batch
    encode, objects compressible or not; a tampered object fails alone."""
    import torch
    from carbonado_amd import device
    n, count = 60_001, 6
    rng = np.random.default_rng(100 + level)
    rows = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(count - 2)]
    rows += [np.zeros(n, np.uint8), np.frombuffer((b"carbonado " * n)[:n], np.uint8)]
    inp = torch.from_numpy(np.stack(rows))
    cap = device._lib.lib().chip_encode_max_len(n)
    enc = torch.zeros((count, cap), dtype=torch.uint8)
    hashes = torch.zeros((count, 32), dtype=torch.uint8)
    olen, info = device.encode_host_batch(level, inp, n, enc, hashes, nslots=2, slice_bytes=2 * n, pubkey=PUB)
    out = torch.zeros((count, n + 64), dtype=torch.uint8)
    pads = [i.padding_len for i in info]
    dlen, st = device.decode_host_batch(level, enc, olen, hashes, pads, out, secret_key=SK, nslots=2,
                                        slice_bytes=2 * n, host_threads=3)
    assert st == [0] * count
    for o in range(count):
        assert dlen[o] == n and out[o, :n].numpy().tobytes() == rows[o].tobytes(), o
    if level & 4:  # flip a content byte of object 2 only
        enc[2, olen[2] // 2] ^= 1
        dlen, st = device.decode_host_batch(level, enc, olen, hashes, pads, out, secret_key=SK, nslots=2,
                                            slice_bytes=2 * n, raise_first=False)
        assert st[2] == 5 and st[:2] == [0, 0] and st[3:] == [0] * (count - 3)
        for o in (0, 1, 3):
            assert out[o, :n].numpy().tobytes() == rows[o].tobytes()


@pytest.mark.parametrize("n", [0, 1, 4096, 12_288, 70_001, (1 << 20) + 1, 3 << 20])
@pytest.mark.parametrize("level", [0, 4, 8, 12])
def test_encode_batch_dev(gpu, level, n):
    """chip_encode_batch_dev (device-resident encode(); Zfec|Bao fused: shards
    written straight into the bao stream, hashed in place) == encode() of the
    oracle per object.  n = 12 KiB gives N = 24 chunks (not a power of two)."""
    import torch
    from carbonado_amd import device
    count = 5
    rng = np.random.default_rng(1000 * level + n % 997)
    stride = (n + 16 + 15) // 16 * 16
    host = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    oenc0, _, _ = O.encode(host[0, :n].tobytes(), level)
    ostride = (len(oenc0) + 48 + 15) // 16 * 16
    out = torch.full((count, ostride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.full((count, 32), 0x5A, dtype=torch.uint8, device="cuda")
    scratch = device.encode_scratch(level, n, count)
    olen, info = device.encode_batch(level, inp, n, out, hashes, scratch)
    torch.cuda.synchronize()
    got, gh = out.cpu().numpy(), hashes.cpu().numpy()
    for o in range(count):
        enc, h, oinfo = O.encode(host[o, :n].tobytes(), level)
        assert olen == len(enc)
        assert got[o, :olen].tobytes() == enc, o
        assert (got[o, olen:] == 0xA5).all(), "bytes past the encoding were written"
        assert gh[o].tobytes() == (h if level & 4 else b"\0" * 32)
    assert info.padding_len == oinfo["padding_len"] and info.output_len == olen


def test_encode_batch_dev_rejects_host_stages(gpu):
    import torch
    from carbonado_amd import device
    from carbonado_amd.error import CarbonadoError
    inp = torch.zeros((2, 4096), dtype=torch.uint8, device="cuda")
    out = torch.zeros((2, 1 << 16), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((2, 32), dtype=torch.uint8, device="cuda")
    for level in (1, 2, 15):
        with pytest.raises(CarbonadoError):
            device.encode_batch(level, inp, 4096, out, hashes, device.encode_scratch(12, 4096, 2))


def test_chip_init_selects_the_process_device(gpu):
    """One process per GPU (bench.py --gpus N): chip_init(d) selects device d
    for every later call; a device that is not a visible gfx950 is refused
    without changing the selection."""
    import torch
    from carbonado_amd import _lib
    L = _lib.lib()
    n = torch.cuda.device_count()
    assert L.chip_init(n) != 0  # one past the last visible device
    assert L.chip_init(n - 1) == 0
    assert L.chip_init(-1) == 0  # keep the current selection
    d = np.random.default_rng(7).integers(0, 256, 50_000, dtype=np.uint8).tobytes()
    import carbonado_amd as ca
    enc, h, _ = ca.encode(b"", d, 12)
    assert (enc, h) == O.encode(d, 12)[:2]
    assert L.chip_init(0) == 0


@pytest.mark.parametrize("n", [0, 1, 4096, 70_001, (1 << 20) + 1, 3 << 20])
@pytest.mark.parametrize("level", [0, 4, 8, 12])
def test_decode_batch_dev_roundtrip(gpu, level, n):
    """chip_decode_batch_dev (device-resident decode(), decoding.rs:80-114)
    inverts chip_encode_batch_dev at every device-only level; at Bao|Zfec only
    the data shards are written, every node still verified.  A flipped byte
    in one object's stream fails that object alone (status 5); its
    neighbours decode."""
    import torch
    from carbonado_amd import device
    count = 4
    rng = np.random.default_rng(7000 + 10 * level + n % 991)
    stride = (n + 16 + 15) // 16 * 16
    host = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    cap = device._lib.lib().chip_encode_max_len(n)
    enc = torch.zeros((count, (cap + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    olen, info = device.encode_batch(level, inp, n, enc, hashes, device.encode_scratch(level, n, count))
    out = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    scratch = device.decode_scratch(level, olen, count)
    dlen = device.decode_batch(level, enc, olen, hashes, info.padding_len, out, status, scratch)
    torch.cuda.synchronize()
    assert dlen == n
    assert status.cpu().tolist() == [0] * count
    got = out.cpu().numpy()
    for o in range(count):
        assert got[o, :n].tobytes() == host[o, :n].tobytes(), o
        assert (got[o, n:] == 0xA5).all(), "bytes past the decoded length were written"
    if level & 4 and n > 0:
        enc[1, olen // 2] ^= 1
        out.fill_(0)
        device.decode_batch(level, enc, olen, hashes, info.padding_len, out, status, scratch)
        torch.cuda.synchronize()
        assert status.cpu().tolist() == [0, 5, 0, 0]
        for o in (0, 2, 3):
            assert out[o, :n].cpu().numpy().tobytes() == host[o, :n].tobytes()


def test_decode_batch_dev_errors(gpu):
    import torch
    from carbonado_amd import device
    from carbonado_amd.error import BaoDecodeError, CarbonadoError, UnevenZfecChunks
    n, count = 50_000, 2
    inp = torch.randint(0, 256, (count, (n + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
    enc = torch.zeros((count, 1 << 18), dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    olen, info = device.encode_batch(12, inp, n, enc, hashes, device.encode_scratch(12, n, count))
    out = torch.zeros((count, 1 << 17), dtype=torch.uint8, device="cuda")
    status = torch.zeros((count,), dtype=torch.int32, device="cuda")
    scratch = device.decode_scratch(12, olen, count)
    with pytest.raises(BaoDecodeError):  # no bao stream has this length (1 KiB: 1032 B, 1025 B: 1097 B)
        device.decode_batch(12, enc, 1040, hashes, info.padding_len, out, status, scratch)
    with pytest.raises(UnevenZfecChunks):  # a bao stream, but of zlen - 1 content bytes
        device.decode_batch(12, enc, olen - 1, hashes, info.padding_len, out, status, scratch)
    with pytest.raises(UnevenZfecChunks):  # zfec-only input that is not 8 shards
        device.decode_batch(8, enc, 8 * 1024 + 3, hashes, 0, out, status, scratch)
    with pytest.raises(CarbonadoError):  # host stages (Snappy/Ecies bits)
        device.decode_batch(15, enc, olen, hashes, info.padding_len, out, status, scratch)
    # a header that disagrees with in_len: the stream of a shorter object, same length
    hdr = enc[0, :8].clone()
    enc[0, :8] = torch.tensor(list((123).to_bytes(8, "little")), dtype=torch.uint8)
    device.decode_batch(12, enc, olen, hashes, info.padding_len, out, status, scratch)
    torch.cuda.synchronize()
    assert status.cpu().tolist() == [5, 0]
    enc[0, :8] = hdr


@pytest.mark.parametrize("cols", [129, 130, 131, 132, 133, 134, 135, 136, 257, 4097])
def test_encode_batch_dev_k13_general_cols(gpu, cols):
    """K13's general path (level-0 CVs to memory, levels 1-3 in the separate
    pass): shards of `cols` chunk-columns, so every offset of a shard
    from the 8-chunk grid (cols % 8 = 1..7, and 0 with zfec padding), 17 to
    513 blocks per object, three objects in
    one launch — every stream and hash == the oracle's encode() level 12."""
    import torch
    from carbonado_amd import device
    count = 3
    rng = np.random.default_rng(cols)
    n = (cols - 1) * 4096 + int(rng.integers(1, 4096))  # zfec padding > 0: the general path
    stride = (n + 255) // 256 * 256
    host = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    oenc0, _, _ = O.encode(host[0, :n].tobytes(), 12)
    ostride = (len(oenc0) + 255) // 256 * 256
    out = torch.full((count, ostride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.full((count, 32), 0x5A, dtype=torch.uint8, device="cuda")
    scratch = device.encode_scratch(12, n, count)
    olen, info = device.encode_batch(12, inp, n, out, hashes, scratch)
    torch.cuda.synchronize()
    assert info.chunk_len == cols * 1024
    got, gh = out.cpu().numpy(), hashes.cpu().numpy()
    for o in range(count):
        enc, h, _ = O.encode(host[o, :n].tobytes(), 12)
        assert olen == len(enc)
        assert got[o, :olen].tobytes() == enc, o
        assert (got[o, olen:] == 0xA5).all()
        assert gh[o].tobytes() == h


@pytest.mark.parametrize("cols,pad,off", [(129, True, 56), (133, True, 8), (136, False, 56), (4097, True, 56),
                                          (256, False, 120)])
def test_encode_batch_dev_stream_offset(gpu, cols, pad, off):
    """Zfec|Bao streams at an 8-B phase in their rows (include/carbonado_hip.h:
    56 mod 64 puts every chunk and node on a 64-B boundary): K13's FULL path
    (cols % 8 == 0, no zfec padding) and general path, the row pitch a 256-B
    multiple plus the offset phase; every stream and hash == the oracle's, no
    byte before the offset or after the stream written."""
    import torch
    from carbonado_amd import device
    count = 3
    rng = np.random.default_rng(cols + off)
    n = (cols - 1) * 4096 + int(rng.integers(1, 4096)) if pad else cols * 4096
    stride = (n + 255) // 256 * 256
    host = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    inp = torch.from_numpy(host).cuda()
    oenc0, _, _ = O.encode(host[0, :n].tobytes(), 12)
    ostride = (off + len(oenc0) + 255) // 256 * 256 + (off % 16)  # the phase repeats in every row
    out = torch.full((count, ostride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.full((count, 32), 0x5A, dtype=torch.uint8, device="cuda")
    scratch = device.encode_scratch(12, n, count)
    olen, info = device.encode_batch(12, inp, n, out, hashes, scratch, out_offset=off)
    torch.cuda.synchronize()
    got, gh = out.cpu().numpy(), hashes.cpu().numpy()
    for o in range(count):
        enc, h, _ = O.encode(host[o, :n].tobytes(), 12)
        assert olen == len(enc)
        assert got[o, off:off + olen].tobytes() == enc, o
        assert (got[o, :off] == 0xA5).all() and (got[o, off + olen:] == 0xA5).all(), o
        assert gh[o].tobytes() == h
    # decode() reads them at that phase (every node verified, the data shards out)
    dec = torch.empty((count, stride), dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    dscr = device.decode_scratch(12, olen, count)
    dlen = device.decode_batch(12, out, olen, hashes, info.padding_len, dec, status, dscr, in_offset=off)
    torch.cuda.synchronize()
    assert dlen == n and int(status.abs().sum()) == 0 and torch.equal(dec[:, :n], inp[:, :n])


def test_encode_batch_dev_stream_offset_refused_where_not_k13(gpu):
    """An 8-B (not 16-B) aligned stream base is refused where the batch does not
    run K13 (small streams take KS): CHIP_ERR_INVALID_ARG, nothing written."""
    import torch
    from carbonado_amd import device
    from carbonado_amd.error import CarbonadoError
    n, count = 4096 * 8, 4  # 32 KiB objects: 64-chunk streams, KS below 64
    inp = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
    out = torch.full((count, 1 << 17), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.zeros((count, 32), dtype=torch.uint8, device="cuda")
    scratch = device.encode_scratch(12, n, count)
    small = 4096 * 3  # 24 KiB: 24-chunk streams (KS)
    with pytest.raises(CarbonadoError):
        device.encode_batch(12, inp[:, :small].contiguous(), small, out, hashes, scratch, out_offset=56)
    torch.cuda.synchronize()
    assert bool((out == 0xA5).all())


@pytest.mark.parametrize("level,n", [(12, 320 << 10), (12, (300 << 10) + 5), (4, (600 << 10) + 77)])
def test_encode_batch_dev_many_small_trees_upper_pass(gpu, level, n):
    """2048 objects whose trees have 65-512 level-3 nodes: levels 4-6 run in
    the levels pass (fused_kernels.hip upper_levels) and the top walk starts
    at level 7 — K13 FULL (320 KiB), general (zfec padding) and the content
    mode (level 4).  Every hash vs the oracle, whole streams of three objects,
    and the batch decode of all (status 0, bytes back)."""
    import torch
    from carbonado_amd import device
    count = 2048
    stride = (n + 255) // 256 * 256
    gen = torch.Generator(device="cuda").manual_seed(n % 4093)
    inp = torch.randint(0, 256, (count, stride), dtype=torch.uint8, device="cuda", generator=gen)
    h_in = inp.cpu().numpy()
    enc0, _, _ = O.encode(h_in[0, :n].tobytes(), level)
    off = device.STREAM_OFFSET
    out = torch.empty((count, (off + len(enc0) + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    olen, info = device.encode_batch(level, inp, n, out, hashes, device.encode_scratch(level, n, count),
                                     out_offset=off)
    torch.cuda.synchronize()
    gh = hashes.cpu().numpy()
    for o in range(count):
        if o in (0, 1031, count - 1):
            enc, h, _ = O.encode(h_in[o, :n].tobytes(), level)
            assert out[o, off:off + olen].cpu().numpy().tobytes() == enc, o
            assert gh[o].tobytes() == h, o
    # every hash: the root of each stream's tree
    for o in range(count):
        assert gh[o].tobytes() == O.encode(h_in[o, :n].tobytes(), level)[1], o
    dec = torch.empty((count, stride), dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    dlen = device.decode_batch(level, out, olen, hashes, info.padding_len, dec, status,
                               device.decode_scratch(level, olen, count), in_offset=off)
    torch.cuda.synchronize()
    assert dlen == n and int(status.abs().sum()) == 0 and torch.equal(dec[:, :n], inp[:, :n])


@pytest.mark.parametrize("level", [5, 7, 9, 11, 13, 15])
def test_decode_key_derived_during_device_work(gpu, level):
    """decode() at Ecies (|Snappy) with Bao and/or Zfec derives the ECIES key from
    the envelope header as the input holds it while the device verifies, and
    decrypts with it only if the verified header equals those bytes
    (api_decode.cpp; host_stages.cpp ecies_decrypt_snap_par).  Round trip at
    1 MiB, a wrong receiver key, and the header's ephemeral key altered inside
    the input: bao refuses the stream, and without bao the tag does."""
    import carbonado_amd as ca
    from carbonado_amd.error import BaoDecodeError, EciesError
    d = np.random.default_rng(level).integers(0, 256, (1 << 20) + 3, dtype=np.uint8).tobytes()
    enc, h, info = ca.encode(PUB, d, level)
    assert ca.decode(SK, h, enc, info.padding_len, level) == d
    with pytest.raises(EciesError):
        ca.decode(H.sha256(b"someone else"), h, enc, info.padding_len, level)
    envelope = O.decode(h, enc, info.padding_len, level & 12)
    pos = enc.find(envelope[:65])
    assert pos >= 0
    bad = bytearray(enc)
    bad[pos + 40] ^= 0x10  # inside the ephemeral public key
    with pytest.raises(BaoDecodeError if level & 4 else EciesError):
        ca.decode(SK, h, bytes(bad), info.padding_len, level)
    assert ca.decode(SK, h, enc, info.padding_len, level) == d  # the stale derived key is not reused


@pytest.mark.parametrize("level", [5, 7, 13, 15])
@pytest.mark.parametrize("n", [1000, 300_000])
def test_verified_stream_with_a_bad_envelope(gpu, level, n):
    """A stream that verifies but whose ECIES envelope does not: the content
    of a level (level & 12) encoding is an envelope with its ephemeral key
    moved off the curve, or with a flipped ciphertext byte; decode() at the
    Ecies level verifies the stream (bao passes), runs the host stages on the
    content meanwhile (no key derived ahead for the off-curve key) and
    returns EciesError (decoding.rs:101-105), for the KS (1000 B) and KM
    (300 kB) routes."""
    import carbonado_amd as ca
    from carbonado_amd.error import EciesError
    d = np.random.default_rng(n + level).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, h, info = ca.encode(PUB, d, level)
    envelope = O.decode(h, enc, info.padding_len, level & 12)
    P = 2**256 - 2**32 - 977
    y = int.from_bytes(envelope[33:65], "big")
    off_curve = envelope[:33] + ((y + 1) % P).to_bytes(32, "big") + envelope[65:]
    flipped = bytearray(envelope)
    flipped[-1] ^= 1
    for bad in (off_curve, bytes(flipped)):
        benc, bh, binfo = ca.encode(b"", bad, level & 12)
        with pytest.raises(EciesError):
            ca.decode(SK, bh, benc, binfo.padding_len, level)
