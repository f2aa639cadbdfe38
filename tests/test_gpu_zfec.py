"""GPU parity: zfec encode/decode kernels (K1/K2) vs the CPU oracle.

Bit-exact byte comparison at sizes the oracle finishes in seconds, edge
sizes (empty, 1 byte, ragged tails, exact multiples), every erasure pattern
of 4-of-8, the 8-of-16 kernel shape, generic fallback shapes, and the full
16 MiB BASELINE object size through erase→decode round trips.
"""
import itertools
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 15, 16, 1023, 1024, 1025, 4095, 4096, 4097, 12289, 65536 + 13, (1 << 20) + 5]


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("n", SIZES)
def test_encode_4of8_matches_oracle(gpu, n):
    from carbonado_amd import encoding
    d = rnd(n, n)
    assert encoding.zfec(d) == O.zfec_encode(d)


@pytest.mark.parametrize("k,m", [(8, 16), (3, 10), (2, 5), (1, 3), (5, 7), (16, 20), (4, 20), (17, 21), (6, 6), (9, 12), (14, 22)])
@pytest.mark.parametrize("n", [1, 5000, 100_003])
def test_encode_other_shapes(gpu, k, m, n):
    from carbonado_amd import encoding
    d = rnd(n, k * 1000 + m + n)
    assert encoding.zfec(d, k, m) == O.zfec_encode(d, k, m)


def test_decode_every_4of8_erasure_pattern(gpu):
    from carbonado_amd import decoding
    d = rnd(50_000, 1)
    z, pad, C = O.zfec_encode(d)
    shards = [z[i * C:(i + 1) * C] for i in range(8)]
    for sub in itertools.combinations(range(8), 4):
        got = decoding.zfec_chunks([shards[i] for i in sub], pad, indices=list(sub))
        assert got == d, sub
    # shares given in scrambled order, and more than k of them
    order = [7, 2, 5, 0, 6]
    assert decoding.zfec_chunks([shards[i] for i in order], pad, indices=order) == d


def test_decode_8of16_random_patterns(gpu):
    from carbonado_amd import decoding
    d = rnd(70_001, 2)
    z, pad, C = O.zfec_encode(d, 8, 16)
    shards = [z[i * C:(i + 1) * C] for i in range(16)]
    r = random.Random(3)
    for _ in range(20):
        sub = sorted(r.sample(range(16), 8))
        assert decoding.zfec_chunks([shards[i] for i in sub], pad, indices=sub, k=8, m=16) == d


def test_decode_too_few_shares(gpu):
    from carbonado_amd import decoding
    from carbonado_amd.error import ZfecError
    z, pad, C = O.zfec_encode(rnd(5000, 4))
    with pytest.raises(ZfecError):
        decoding.zfec_chunks([z[:C], z[C:2 * C], z[2 * C:3 * C]], pad, indices=[0, 1, 2])
    with pytest.raises(ZfecError):  # duplicates do not count twice
        decoding.zfec_chunks([z[:C]] * 4, pad, indices=[0, 0, 0, 0])


@pytest.mark.parametrize("n", SIZES)
def test_positional_decode_roundtrip(gpu, n):
    """decoding.rs:34-51 (positional indices, all shards present)."""
    from carbonado_amd import decoding, encoding
    d = rnd(n, n + 7)
    z, pad, C = encoding.zfec(d)
    assert decoding.zfec(z, pad) == d == O.zfec_decode(z, pad)


def test_reference_positional_quirk(gpu):
    """With data shard 0 lost, position-numbered survivors (decoding.rs:24-25,
    as scrub() passes them) decode to the wrong bytes in the reference; the
    explicit-index entry point recovers the data."""
    from carbonado_amd import decoding
    d = rnd(20_000, 5)
    z, pad, C = O.zfec_encode(d)
    shards = [z[i * C:(i + 1) * C] for i in range(8)]
    surv = [shards[i] for i in range(1, 8)]
    assert decoding.zfec_chunks(surv, pad) != d  # positional mislabel
    assert decoding.zfec_chunks(surv, pad, indices=list(range(1, 8))) == d


def test_batch_device_api_ragged(gpu):
    import torch
    from carbonado_amd import device
    n, count = 1_000_003, 6
    stride = (n + 15) // 16 * 16
    host = np.stack([np.frombuffer(rnd(n, 100 + o), np.uint8) for o in range(count)])
    inp = torch.zeros((count, stride), dtype=torch.uint8, device="cuda")
    inp[:, :n] = torch.from_numpy(host).cuda()
    pad, C = O.calc_padding_len(n)
    out = torch.empty((count, 8 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for o in range(count):
        assert got[o].tobytes() == O.zfec_encode(host[o].tobytes())[0], o
    # erasure decode of the same batch, two data shards lost
    dec = torch.empty((count, 4 * C), dtype=torch.uint8, device="cuda")
    device.zfec_decode_batch(out, C, [0, 3, 4, 5, 6, 7], dec)
    torch.cuda.synchronize()
    d = dec.cpu().numpy()
    for o in range(count):
        assert d[o, :n].tobytes() == host[o].tobytes()


def test_full_size_16mib_objects(gpu):
    """BASELINE cfg2/cfg3 object size: 16 MiB objects, 4 of them; parity of
    object 0 bit-exact vs the oracle; every object survives the cfg3 erasure
    (shards 1 and 2 dropped) and the worst pattern {0,1,2,3}."""
    import torch
    from carbonado_amd import device
    n, count = 16 << 20, 4
    gen = torch.Generator(device="cuda").manual_seed(11)
    inp = torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=gen)
    out = torch.empty((count, 2 * n), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, n, out)
    torch.cuda.synchronize()
    obj0 = inp[0].cpu().numpy().tobytes()
    assert out[0].cpu().numpy().tobytes() == O.zfec_encode(obj0)[0]
    C = n // 4
    for keep in ([0, 3, 4, 5, 6, 7], [4, 5, 6, 7]):
        dec = torch.empty((count, n), dtype=torch.uint8, device="cuda")
        device.zfec_decode_batch(out, C, keep, dec)
        torch.cuda.synchronize()
        assert torch.equal(dec, inp)


@pytest.mark.parametrize("n", [1, 15, 17, 4093, 1_000_003])
def test_batch_bytes_past_n_read_as_zero(gpu, n):
    """Bytes of an input row beyond n must count as zero padding
    (encoding.rs:53-55) even when the row holds garbage there: K1's tail load
    masks the partially valid 16-B block."""
    import torch
    from carbonado_amd import device
    count = 3
    stride = (n + 15) // 16 * 16 + 32
    host = np.stack([np.frombuffer(rnd(n, 700 + o), np.uint8) for o in range(count)])
    inp = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    inp[:, :n] = torch.from_numpy(host).cuda()
    pad, C = O.calc_padding_len(n)
    out = torch.empty((count, 8 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for o in range(count):
        assert got[o].tobytes() == O.zfec_encode(host[o].tobytes())[0], o


def test_batch_misaligned_pointer_rejected(gpu):
    import ctypes
    import torch
    from carbonado_amd import _lib
    from carbonado_amd.error import InvalidArgument
    from carbonado_amd._buf import check
    n = 4096
    inp = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    lib = _lib.lib()
    p_in, p_out = inp.data_ptr(), out.data_ptr()
    assert p_in % 16 == 0 and p_out % 16 == 0
    for a, b in ((p_in + 1, p_out), (p_in, p_out + 8)):
        with pytest.raises(InvalidArgument):
            check(lib.chip_zfec_encode_batch_dev(4, 8, ctypes.c_void_p(a), n + 16, n, 1, ctypes.c_void_p(b),
                                                 2 * n, None))
    idx = (ctypes.c_uint32 * 4)(4, 5, 6, 7)
    with pytest.raises(InvalidArgument):
        check(lib.chip_zfec_decode_batch_dev(4, 8, ctypes.c_void_p(p_out + 4), 2 * n, n // 4, idx, 4, 1,
                                             ctypes.c_void_p(p_in), n, None))


@pytest.mark.parametrize("k,m,n", [(4, 8, 16 << 20), (4, 8, 1_000_003), (8, 16, 100_000), (4, 8, 5)])
def test_batch_in_place_aliased_data_shards(gpu, k, m, n):
    """d_out == d_in: the data shards stay where they are, only parity is
    written and the padding tail is zeroed (SURVEY.md 8d 'aliased')."""
    import torch
    from carbonado_amd import device
    count = 2
    pad, C = O.calc_padding_len(n, k)
    buf = torch.full((count, m * C), 0x5A, dtype=torch.uint8, device="cuda")  # garbage everywhere
    host = [np.frombuffer(rnd(n, 900 + o), np.uint8) for o in range(count)]
    for o in range(count):
        buf[o, :n] = torch.from_numpy(host[o]).cuda()
    device.zfec_encode_batch(buf, n, buf, k, m)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for o in range(count):
        assert got[o].tobytes() == O.zfec_encode(host[o].tobytes(), k, m)[0], o


@pytest.mark.parametrize("k,m,n", [(4, 8, (1 << 20) + 5), (4, 8, 16 << 20), (8, 16, (1 << 20) + 5)])
def test_hbm_pattern_probe_writes_its_pattern(gpu, k, m, n):
    """chip_hbm_pattern_batch_dev (bench.py's box ceiling) runs the encode's
    memory pattern: data shards copied, computed row q = the XOR of the k data
    shards with every byte XOR q — every output byte written (the same tiles
    as the encode)."""
    import torch
    from carbonado_amd import device
    count = 3
    row = (n + 15) // 16 * 16  # batch rows are 16-B aligned; bytes past n read as zero
    inp = torch.randint(0, 256, (count, row), dtype=torch.uint8, device="cuda")
    C = gpu.chip_zfec_encoded_len(n, k, m) // m
    out = torch.full((count, m * C), 0xA5, dtype=torch.uint8, device="cuda")
    device.hbm_pattern_batch(inp, n, out, k, m)
    torch.cuda.synchronize()
    padded = torch.zeros((count, k * C), dtype=torch.uint8, device="cuda")
    padded[:, :n] = inp[:, :n]
    sh = padded.view(count, k, C)
    got = out.view(count, m, C)
    assert torch.equal(got[:, :k], sh)
    x = sh[:, 0].clone()
    for j in range(1, k):
        x ^= sh[:, j]
    for q in range(m - k):
        assert torch.equal(got[:, k + q], x ^ q), q


def test_hbm_pattern_probe_refuses_other_shapes(gpu):
    import torch
    from carbonado_amd import _lib
    inp = torch.zeros((1, 4096), dtype=torch.uint8, device="cuda")
    out = torch.zeros((1, 8192), dtype=torch.uint8, device="cuda")
    L = _lib.lib()
    assert L.chip_hbm_pattern_batch_dev(3, 6, inp.data_ptr(), 4096, 4096, 1, out.data_ptr(), 8192, None) == 7
    assert L.chip_hbm_pattern_batch_dev(4, 8, inp.data_ptr(), 4096, 4096, 1, inp.data_ptr(), 4096, None) == 1
