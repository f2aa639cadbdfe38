"""GPU: the single-object calls copy pageable host buffers through the pinned
staging ring and pinned buffers directly (api_host_copy.cpp h2d/d2h); every
combination gives the oracle's bytes, including buffers that wrap the 4 x 4
MiB ring several times, odd lengths and unaligned addresses."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _pinned(a: np.ndarray) -> np.ndarray:
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()


@pytest.mark.parametrize("n", [300_000, (4 << 20) + 17, (20 << 20) + 5])
def test_encode_decode_pinned_and_pageable(gpu, n):
    import carbonado_amd as ca
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    ref, href, _ = O.encode(d.tobytes(), 12)
    e1, h1, info = ca.encode(b"", d, 12)  # pageable: staged
    e2, h2, _ = ca.encode(b"", _pinned(d), 12)  # pinned: direct
    assert e1 == ref and h1 == href
    assert e2 == ref and h2 == href
    enc = np.frombuffer(ref, np.uint8)
    assert ca.decode(b"", href, enc, info.padding_len, 12) == d.tobytes()
    assert ca.decode(b"", href, _pinned(enc), info.padding_len, 12) == d.tobytes()


def test_unaligned_pageable_buffers(gpu):
    """Input and output at odd addresses (the ring copies are plain memcpy)."""
    import carbonado_amd as ca
    from carbonado_amd import _lib
    from carbonado_amd._buf import ptr
    n = (6 << 20) + 3
    raw = np.random.default_rng(7).integers(0, 256, n + 1, dtype=np.uint8)
    d = raw[1:]  # address + 1
    ref, href, _ = O.encode(d.tobytes(), 12)
    assert ca.encode(b"", d, 12)[0] == ref
    out = np.empty(len(ref) + 3, np.uint8)
    olen = ctypes.c_uint64()
    h = np.frombuffer(href, np.uint8)
    enc = np.frombuffer(ref, np.uint8)
    L = _lib.lib()
    # bao decode of the whole level-12 stream into out[3:] (content = the zfec shards)
    rc = L.chip_bao_decode(ptr(enc), enc.size, ptr(h), 32, ctypes.c_void_p(out.ctypes.data + 3), len(ref),
                           ctypes.byref(olen))
    assert rc == 0
    assert out[3:3 + olen.value].tobytes() == O.zfec_encode(d.tobytes())[0]


def test_hasher_pageable_and_pinned_appends(gpu):
    """BaoHasher appends alternating pageable and pinned pieces (staged ones
    return before their DMA completes; the ring must not be overwritten)."""
    from carbonado_amd.utils import BaoHasher
    rng = np.random.default_rng(11)
    pieces = [rng.integers(0, 256, s, dtype=np.uint8) for s in (5 << 20, 1 << 20, 300_000, 9 << 20, 17, 4 << 20)]
    h = BaoHasher()
    for i, p in enumerate(pieces):
        h.update(_pinned(p) if i % 2 else p)
    allb = b"".join(p.tobytes() for p in pieces)
    assert bytes(h.finalize()) == O.blake3(allb)
    assert h.read_all() == O.bao_encode(allb)[0]


def test_host_topology_ring_and_workers_on_the_gpu_node(gpu):
    """chip_host_topology after a staged copy: the ring exists, and with NUMA
    placement on (the default) the ring's pages and every copy worker that
    has run sit on the GPU's node whenever the process may use its CPUs."""
    import carbonado_amd as ca
    from carbonado_amd.device import host_topology
    d = np.random.default_rng(3).integers(0, 256, 24 << 20, dtype=np.uint8)
    enc, h, info = ca.encode(b"", d, 12)  # pageable in and out: through the ring
    t = host_topology()
    for key in ("gpu_pci", "gpu_node", "ring_node", "copy_workers", "copy_workers_pinned",
                "copy_workers_by_last_cpu_node", "numa_placement"):
        assert key in t, t
    assert t["ring_node"] >= 0, t
    if t["numa_placement"] and t["gpu_node"] >= 0 and t["gpu_local_cpus_allowed"] > 0:
        assert t["copy_workers_pinned"], t
        assert t["ring_node"] == t["gpu_node"], t
        ran = {k: v for k, v in t["copy_workers_by_last_cpu_node"].items() if k != "idle"}
        assert set(ran) <= {str(t["gpu_node"])}, t
