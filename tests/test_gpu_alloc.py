"""GPU: the batch-buffer allocator (chip_device_alloc / chip_torch_alloc and
carbonado_amd.device.empty_batch): physically contiguous HBM usable by the
batch entry points like any other device memory."""
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
    assert L.chip_device_free(p) == 0
    assert L.chip_device_free(None) == 0


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
