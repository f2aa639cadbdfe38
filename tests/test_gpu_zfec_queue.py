"""GPU: the dynamic per-XCD run queue of K1/K2 (zfec_device.hpp QueueIter,
MAP 6).  Workgroups take runs of tiles with one atomic each and take other
XCDs' runs once their own share is done; the last workgroup resets the
counters.  Every tile must be written exactly once in every launch: large and
tiny batches, launch after launch on one stream (the reset), and two streams
at once (each stream has its own counters)."""
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 16 << 20


def _rand(shape, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, shape, dtype=torch.uint8, device="cuda", generator=g)


def test_large_batch_encode_decode_exact(gpu):
    import torch
    from carbonado_amd import device
    count = 67  # > 1 GiB of input, not a multiple of 8
    inp = _rand((count, N), 5)
    enc = torch.zeros((count, 2 * N), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, enc, 4, 8)
    torch.cuda.synchronize()
    for o in (0, 7, 8, 33, 47, 66):
        assert enc[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes())[0], o
    out = torch.zeros((count, N), dtype=torch.uint8, device="cuda")
    device.zfec_decode_batch(enc, N // 4, [0, 3, 4, 5, 6, 7], out, 4, 8)
    torch.cuda.synchronize()
    assert torch.equal(out, inp)


def test_repeated_launches_same_stream(gpu):
    """The counters left by one launch must be zero for the next: ten launches
    back to back on one stream give the same bytes."""
    import torch
    from carbonado_amd import device
    count, n = 24, (2 << 20) + 4096
    inp = _rand((count, n), 11)
    C = O.calc_padding_len(n)[1]
    ref = torch.zeros((count, 8 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, n, ref, 4, 8)
    for _ in range(10):
        out = torch.zeros_like(ref)
        device.zfec_encode_batch(inp, n, out, 4, 8)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    assert ref[5].cpu().numpy().tobytes() == O.zfec_encode(inp[5].cpu().numpy().tobytes())[0]


def test_two_streams_at_once(gpu):
    import torch
    from carbonado_amd import device
    count = 40
    a, b = _rand((count, N), 21), _rand((count, N), 22)
    ra = torch.zeros((count, 2 * N), dtype=torch.uint8, device="cuda")
    rb = torch.zeros_like(ra)
    device.zfec_encode_batch(a, N, ra, 4, 8)
    device.zfec_encode_batch(b, N, rb, 4, 8)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    oa, ob = torch.zeros_like(ra), torch.zeros_like(rb)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        device.zfec_encode_batch(a, N, oa, 4, 8)
    with torch.cuda.stream(s2):
        device.zfec_encode_batch(b, N, ob, 4, 8)
    torch.cuda.synchronize()
    assert torch.equal(oa, ra) and torch.equal(ob, rb)


@pytest.mark.parametrize("count,n", [(1, 4096), (1, 100_003), (3, 1 << 20), (9, 333_333), (17, 65536)])
def test_small_batches(gpu, count, n):
    """Fewer runs than workgroups (grids smaller than 8, most workgroups find
    no run) and ragged tails."""
    import torch
    from carbonado_amd import device
    inp = _rand((count, (n + 15) // 16 * 16), 100 + count)  # rows 16-B aligned (the C-ABI's contract)
    C = O.calc_padding_len(n)[1]
    out = torch.zeros((count, 8 * C), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, n, out, 4, 8)
    torch.cuda.synchronize()
    for o in range(count):
        assert out[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o, :n].cpu().numpy().tobytes())[0], o


def test_8of16_queue_exact(gpu):
    import torch
    from carbonado_amd import device
    count = 20
    inp = _rand((count, N), 31)
    enc = torch.zeros((count, 2 * N), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, enc, 8, 16)
    torch.cuda.synchronize()
    for o in (0, 9, 19):
        assert enc[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes(), 8, 16)[0], o
