"""GPU: the batch-buffer allocator (chip_device_alloc / chip_torch_alloc and
carbonado_amd.device.empty_batch).  From 1 GiB up it is class-balanced
(hbm_alloc.hpp: shuffled 8 MiB pieces behind a fresh virtual range), below
that physically contiguous; both are usable by the batch entry points like
any other device memory."""
import ctypes

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_device_alloc_roundtrip(gpu):
    from carbonado_amd import _lib
    L = _lib.lib()
    p = ctypes.c_void_p()
    assert L.chip_device_alloc(3 << 30, ctypes.byref(p)) == 0 and p.value
    assert p.value % 256 == 0
    found, used, secs = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_double()
    assert L.chip_device_alloc_info(p, ctypes.byref(found), ctypes.byref(used), ctypes.byref(secs)) == 0
    assert 1 <= used.value <= found.value and secs.value > 0
    assert L.chip_device_free(p) == 0
    assert L.chip_device_free(None) == 0
    q = ctypes.c_void_p()
    assert L.chip_device_alloc(1 << 20, ctypes.byref(q)) == 0 and q.value  # small: contiguous / hipMalloc
    assert L.chip_device_alloc_info(q, None, None, None) == 1  # CHIP_ERR_INVALID_ARG
    assert L.chip_device_free(q) == 0


def test_balanced_buffers_encode_exactly(gpu):
    """Two class-balanced buffers (1.1 GiB in, 2.2 GiB out, allocated, freed
    and allocated again: a fresh virtual range each time) carry a bit-exact
    encode + decode."""
    import torch
    from carbonado_amd import _lib, device
    n, count = 16 << 20, 70
    for rnd in range(2):
        inp = device.empty_batch((count, n))
        g = torch.Generator(device="cuda").manual_seed(40 + rnd)
        inp.copy_(torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=g))
        out = device.empty_batch((count, 2 * n))
        device.zfec_encode_batch(inp, n, out, 4, 8)
        torch.cuda.synchronize()
        for o in (0, 35, count - 1):
            assert out[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes())[0], (rnd, o)
        back = torch.zeros((count, n), dtype=torch.uint8, device="cuda")
        device.zfec_decode_batch(out, n // 4, [0, 3, 4, 5, 6, 7], back, 4, 8)
        torch.cuda.synchronize()
        assert torch.equal(back, inp)
        del inp, out, back
        torch.cuda.empty_cache()
        torch.cuda.synchronize()


def test_empty_batch_encodes_exactly(gpu):
    import torch
    from carbonado_amd import device
    n, count = (1 << 20) + 4096, 6
    g = torch.Generator(device="cuda").manual_seed(3)
    inp = device.empty_batch((count, n))
    inp.copy_(torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=g))
    C = O.calc_padding_len(n)[1]
    out = device.empty_batch((count, 8 * C))
    device.zfec_encode_batch(inp, n, out, 4, 8)
    torch.cuda.synchronize()
    for o in (0, count - 1):
        assert out[o].cpu().numpy().tobytes() == O.zfec_encode(inp[o].cpu().numpy().tobytes())[0]
    del inp, out
    torch.cuda.synchronize()
