"""GPU: the run-time choice of the zfec 4-of-8 schedule (zfec_kernels.hip
k4_tune).  The first launch of >= 1 GiB runs two slices of count/8 objects
per candidate schedule, interleaved, then the rest of the batch with the
fastest; every object of every slice stays bit-exact."""
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 16 << 20
COUNT = 67  # > 1 GiB of input (the smallest batch that tunes), not a multiple of 8
# slices of 8 objects: S0 S1 S2 S0 S1 S2 (4-of-8 has three candidates), then the 19-object remainder
CHECK = (0, 7, 8, 16, 24, 32, 40, 47, 48, 66)


def test_encode_then_decode_tune_and_stay_exact(gpu):
    import torch
    from carbonado_amd import _lib, device
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(5)
    inp = torch.randint(0, 256, (COUNT, N), dtype=torch.uint8, device="cuda", generator=g)
    enc = torch.empty((COUNT, 2 * N), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, enc, 4, 8)
    torch.cuda.synchronize()
    assert L.chip_zfec_k4_schedule(8) in (0, 1, 2)
    for o in CHECK:
        assert enc[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes())[0], o

    # decode with data shards 1 and 2 lost: 4 output shards per column
    C = N // 4
    keep = [0, 3, 4, 5, 6, 7]
    out = torch.empty((COUNT, N), dtype=torch.uint8, device="cuda")
    device.zfec_decode_batch(enc, C, keep, out, 4, 8)
    torch.cuda.synchronize()
    assert L.chip_zfec_k4_schedule(4) in (0, 1, 2)
    for o in CHECK:
        assert torch.equal(out[o], inp[o]), o


def test_two_stream_split_is_exact(gpu, monkeypatch):
    """A >= 2 GiB batch: the first one times its quarters as one launch and as
    two concurrent halves (auto), CHIP_ZF_SPLIT=1 forces the halves; encode and
    decode stay bit-exact either way."""
    import torch
    from carbonado_amd import device
    count = 160  # 2.5 GiB of input
    g = torch.Generator(device="cuda").manual_seed(9)
    inp = torch.randint(0, 256, (count, N), dtype=torch.uint8, device="cuda", generator=g)
    ref = torch.empty((count, 2 * N), dtype=torch.uint8, device="cuda")
    device.zfec_encode_batch(inp, N, ref, 4, 8)  # unsplit (and tunes the schedule if needed)
    monkeypatch.setenv("CHIP_ZF_SPLIT", "1")
    enc = torch.zeros_like(ref)
    device.zfec_encode_batch(inp, N, enc, 4, 8)
    torch.cuda.synchronize()
    assert torch.equal(enc, ref)
    out = torch.zeros((count, N), dtype=torch.uint8, device="cuda")
    device.zfec_decode_batch(enc, N // 4, [0, 3, 4, 5, 6, 7], out, 4, 8)
    torch.cuda.synchronize()
    assert torch.equal(out, inp)
    # the unsplit reference itself went through the split auto-tuning (quarters run
    # single, split, single, split) when the schedule was already known: one object
    # of each quarter against the oracle
    for o in (0, 41, 82, 123, count - 1):
        assert ref[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes())[0], o
