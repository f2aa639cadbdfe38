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


def test_concurrent_kernel_families_on_neighbouring_streams(gpu):
    """Two host threads (each with its own stream and run-queue block)
    alternate K1 zfec encodes, K13 content-mode bao encodes and K3 verify-
    decodes, so persistent launches of different families overlap on
    neighbouring streams; every result stays bit-exact.  (The queue blocks
    were once 2 KiB while K13 / K3 kept their counters at words 512-672,
    i.e. in the next stream's K1 counters.)"""
    import threading
    import numpy as np
    import carbonado_amd as ca
    rng = np.random.default_rng(11)
    zd = rng.integers(0, 256, 6 << 20, dtype=np.uint8).tobytes()
    bd = rng.integers(0, 256, (2 << 20) + 4096, dtype=np.uint8).tobytes()
    z_want = O.zfec_encode(zd)[0]
    b_want, b_hash = O.bao_encode(bd)
    errors = []

    def work(tid):
        try:
            for i in range(24):
                op = (i + tid) % 3
                if op == 0:
                    assert ca.encoding.zfec(zd)[0] == z_want
                elif op == 1:
                    assert ca.encoding.bao(bd) == (b_want, b_hash)
                else:
                    assert ca.decoding.bao(b_want, b_hash) == bd
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((tid, repr(e)[:200]))
    ts = [threading.Thread(target=work, args=(t,)) for t in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_concurrent_streams_k13_beside_k1(gpu):
    """Back-to-back batches on two streams registered one after the other:
    K13 content-mode bao encodes on the first, K1 zfec encodes on the second,
    so the two persistent kernels run side by side with neighbouring run-queue
    blocks.  Every round bit-exact (round 0 against the oracle, the others
    against round 0)."""
    import torch
    from carbonado_amd import _lib, device
    L = _lib.lib()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    nb, cb, nz, cz, R = 4 << 20, 16, 16 << 20, 8, 6
    bin_ = _rand((cb, nb), 21)
    zin = _rand((cz, nz), 22)
    bstride = (L.chip_bao_encoded_len(nb) + 15) // 16 * 16
    bouts = [torch.zeros((cb, bstride), dtype=torch.uint8, device="cuda") for _ in range(R)]
    bh = [torch.zeros((cb, 32), dtype=torch.uint8, device="cuda") for _ in range(R)]
    zouts = [torch.zeros((cz, 2 * nz), dtype=torch.uint8, device="cuda") for _ in range(R)]
    bscr = device.bao_scratch(nb, cb)
    torch.cuda.synchronize()
    for r in range(R):  # stream sa first: its queue block precedes sb's
        with torch.cuda.stream(sa):
            device.bao_encode_batch(bin_, nb, bouts[r], bh[r], bscr)
        with torch.cuda.stream(sb):
            device.zfec_encode_batch(zin, nz, zouts[r], 4, 8)
    torch.cuda.synchronize()
    blen = L.chip_bao_encoded_len(nb)
    enc0, h0 = O.bao_encode(bin_[3].cpu().numpy().tobytes())
    assert bouts[0][3, :blen].cpu().numpy().tobytes() == enc0 and bh[0][3].cpu().numpy().tobytes() == h0
    assert zouts[0][5].cpu().numpy().tobytes() == O.zfec_encode(zin[5].cpu().numpy().tobytes())[0]
    for r in range(1, R):
        assert torch.equal(bouts[r], bouts[0]) and torch.equal(bh[r], bh[0]), r
        assert torch.equal(zouts[r], zouts[0]), r


def test_queue_blocks_never_shared_past_pool(gpu):
    """300 distinct caller streams (more than one pool of 256 blocks; created
    with hipStreamCreate: torch.cuda.Stream() hands out a pool of 32) each get
    a run-queue block of their own; then K13 content-mode bao batches on
    stream 1 run concurrently with K1 zfec batches on stream 257, the pair a
    wrapping pool (nx % 256) used to give the same block.  Bit-exact against
    the oracle / round 0."""
    import ctypes
    import torch
    from carbonado_amd import _lib, device
    L = _lib.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    raw = []
    for _ in range(300):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        raw.append(s)
    try:
        blocks = []
        for s in raw:
            a = ctypes.c_uint64()
            assert L.chip_stream_queue_block(s, ctypes.byref(a)) == 0
            blocks.append(a.value)
        own = ctypes.c_uint64()
        assert L.chip_stream_queue_block(None, ctypes.byref(own)) == 0
        assert len(set(blocks + [own.value])) == 301
        again = ctypes.c_uint64()  # stable per stream
        L.chip_stream_queue_block(raw[7], ctypes.byref(again))
        assert again.value == blocks[7]
        sa, sb = torch.cuda.ExternalStream(raw[1].value), torch.cuda.ExternalStream(raw[257].value)
        nb, cb, nz, cz, R = 4 << 20, 16, 16 << 20, 8, 4
        bin_ = _rand((cb, nb), 41)
        zin = _rand((cz, nz), 42)
        bstride = (L.chip_bao_encoded_len(nb) + 15) // 16 * 16
        bouts = [torch.zeros((cb, bstride), dtype=torch.uint8, device="cuda") for _ in range(R)]
        bh = [torch.zeros((cb, 32), dtype=torch.uint8, device="cuda") for _ in range(R)]
        zouts = [torch.zeros((cz, 2 * nz), dtype=torch.uint8, device="cuda") for _ in range(R)]
        bscr = device.bao_scratch(nb, cb)
        torch.cuda.synchronize()
        for r in range(R):
            with torch.cuda.stream(sa):
                device.bao_encode_batch(bin_, nb, bouts[r], bh[r], bscr)
            with torch.cuda.stream(sb):
                device.zfec_encode_batch(zin, nz, zouts[r], 4, 8)
        sa.synchronize()
        sb.synchronize()
        torch.cuda.synchronize()
        blen = L.chip_bao_encoded_len(nb)
        enc0, h0 = O.bao_encode(bin_[9].cpu().numpy().tobytes())
        assert bouts[0][9, :blen].cpu().numpy().tobytes() == enc0 and bh[0][9].cpu().numpy().tobytes() == h0
        assert zouts[0][2].cpu().numpy().tobytes() == O.zfec_encode(zin[2].cpu().numpy().tobytes())[0]
        for r in range(1, R):
            assert torch.equal(bouts[r], bouts[0]) and torch.equal(bh[r], bh[0]), r
            assert torch.equal(zouts[r], zouts[0]), r
    finally:
        torch.cuda.synchronize()
        for s in raw:
            hip.hipStreamSynchronize(s)
            hip.hipStreamDestroy(s)
