"""GPU parity: streaming BaoHasher (utils.rs:104-137) vs the oracle.

update() in arbitrary pieces must give the same root hash (BLAKE3 of the
concatenation) and the same combined encoding as one-shot bao encode;
concurrent updates are serialised by the hasher's lock (the reference uses an
RwLock around bao's Encoder)."""
import threading

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _pieces(total, seed):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
    cuts = sorted(rng.integers(0, total + 1, 7).tolist()) if total else []
    parts, prev = [], 0
    for c in cuts + [total]:
        parts.append(data[prev:c])
        prev = c
    return data, parts


@pytest.mark.parametrize("total", [0, 1, 1023, 1024, 1025, 8191, 65536, 65537, 70_000, 131072, 131073,
                                   (64 << 10) * 65, (3 << 20) + 17])
def test_hasher_matches_oneshot(gpu, total):
    from carbonado_amd.utils import BaoHasher
    data, parts = _pieces(total, total)
    h = BaoHasher.new()
    for p in parts:
        h.update(p)
    assert len(h) == total
    digest = h.finalize()
    enc, oh = O.bao_encode(data)
    assert digest == oh == O.blake3(data)
    assert str(digest) == oh.hex() and digest.to_bytes() == oh
    assert h.read_all() == enc
    assert h.finalize() == digest  # idempotent


def test_hasher_growth_many_small_updates(gpu):
    from carbonado_amd.utils import BaoHasher
    rng = np.random.default_rng(5)
    chunks = [rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes() for _ in range(400)]
    h = BaoHasher()
    for c in chunks:
        h.update(c)
    data = b"".join(chunks)
    assert h.finalize() == O.blake3(data)
    assert h.read_all() == O.bao_encode(data)[0]


def test_hasher_concurrent_updates(gpu):
    """4 threads append identical blocks: any serialisation gives the same bytes."""
    from carbonado_amd.utils import BaoHasher
    block = np.random.default_rng(9).integers(0, 256, 3000, dtype=np.uint8).tobytes()
    h = BaoHasher()

    def work():
        for _ in range(25):
            h.update(block)
    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(h) == 100 * len(block)
    assert h.finalize() == O.blake3(block * 100)


def test_hasher_state_errors(gpu):
    from carbonado_amd.error import InvalidArgument
    from carbonado_amd.utils import BaoHasher
    h = BaoHasher()
    h.update(b"abc")
    with pytest.raises(InvalidArgument):
        h.read_all()  # before finalize
    h.finalize()
    with pytest.raises(InvalidArgument):
        h.update(b"more")  # bao's Encoder cannot take bytes after finalize


def test_hasher_churn_recycles_queue_blocks(gpu):
    """Hundreds of hashers, each with its own stream and (once it runs a
    persistent kernel) its own run-queue block, created and freed one after
    another past the 256-block pool: blocks of freed streams are reused, and
    every digest stays exact while a long-lived stream (this thread's K1
    encodes) keeps its own block."""
    import gc
    import carbonado_amd as ca
    from carbonado_amd.utils import BaoHasher
    data = np.random.default_rng(9).integers(0, 256, (1 << 20) + 5, dtype=np.uint8).tobytes()
    want = O.blake3(data)
    zd = data[: 3 << 20] if len(data) >= 3 << 20 else data * 3
    z_want = O.zfec_encode(zd)[0]
    for i in range(300):
        h = BaoHasher.new()
        h.update(data)
        assert h.finalize() == want, i
        del h
        if i % 50 == 0:
            gc.collect()
            assert ca.encoding.zfec(zd)[0] == z_want


@pytest.mark.parametrize("piece,total", [(4 << 20, (16 << 20) + 5), (65536, (2 << 20)), (65537, (2 << 20) + 999),
                                         (1000, 300_000), (1 << 20, 64 << 20), ((3 << 20) + 7, (40 << 20) + 3),
                                         (32 << 20, (96 << 20) + 65536)])
def test_hasher_incremental_appends(gpu, piece, total):
    """Appends of fixed size at chunk- and unit-misaligned boundaries: the
    chunks hashed during update() (64-chunk units with bytes past them, one
    launch per 32 MiB of them) plus the ones finalize() hashes give the
    one-shot stream and hash."""
    from carbonado_amd.utils import BaoHasher
    rng = np.random.default_rng(piece ^ total)
    data = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
    h = BaoHasher()
    for off in range(0, total, piece):
        h.update(data[off:off + piece])
    enc, oh = O.bao_encode(data)
    assert h.finalize() == oh
    assert h.read_all() == enc


def test_hasher_incremental_pinned_appends(gpu):
    """Pinned (direct-copy) appends of a torch buffer, 4 MiB each, unit
    boundaries inside appends; then the same hasher's stream vs the oracle."""
    import torch
    from carbonado_amd.utils import BaoHasher
    total = (40 << 20) + 4097  # past the 32 MiB of units that trigger hashing during update()
    src = torch.randint(0, 256, (total,), dtype=torch.uint8).pin_memory()
    h = BaoHasher()
    piece = (4 << 20) - 3
    for off in range(0, total, piece):
        h.update(src[off:off + piece].numpy())
    data = src.numpy().tobytes()
    enc, oh = O.bao_encode(data)
    assert h.finalize() == oh
    assert h.read_all() == enc


def test_hasher_grows_in_place_across_pieces(gpu):
    """Round 4: the content grows behind a reserved VA range (8 MiB ... 1 GiB
    physical pieces, no copy, no device sync).  600 MiB in 8 MiB + 13-byte
    appends crosses several piece boundaries while update()-time hashing of
    the earlier units is in flight; hash and stream equal the oracle's."""
    from carbonado_amd.utils import BaoHasher
    rng = np.random.default_rng(41)
    data = rng.integers(0, 256, 600 << 20, dtype=np.uint8)
    h = BaoHasher()
    step = (8 << 20) + 13
    for off in range(0, data.size, step):
        h.update(data[off:off + step])
    raw = data.tobytes()
    assert h.finalize() == O.blake3(raw)
    enc = h.read_all()
    assert len(enc) == O.lib().orc_bao_encoded_len(len(raw))
    assert O.blake3(enc) == O.blake3(O.bao_encode(raw)[0])


def test_hasher_outgrows_its_va_range(gpu, monkeypatch):
    """A hasher whose content outgrows its first VA range (1 GiB:
    CHIP_HASHER_VA_MIB, the default too; ranges are whole GiB) moves once
    into a fresh range 4x its need (one device copy of the bytes so far) and
    keeps every byte."""
    from carbonado_amd.utils import BaoHasher
    monkeypatch.setenv("CHIP_HASHER_VA_MIB", "1024")
    rng = np.random.default_rng(43)
    data = rng.integers(0, 256, (1 << 30) + (200 << 20) + 7, dtype=np.uint8)
    h = BaoHasher()  # the reserve is read when the hasher is made
    monkeypatch.delenv("CHIP_HASHER_VA_MIB")
    step = 64 << 20
    for off in range(0, data.size, step):
        h.update(data[off:off + step])
    assert h.finalize() == O.blake3(data.tobytes())


def test_hasher_reuses_a_freed_hashers_resources(gpu):
    """A freed hasher's streams and grown buffers go to the next one (one
    spare, CHIP_HASHER_CACHE=0 disables it).  Large, then small, then
    larger: every hasher starts empty and gives the oracle's hash and
    stream, whatever the previous one left in the reused buffers."""
    import gc
    from carbonado_amd.utils import BaoHasher
    rng = np.random.default_rng(47)
    for total in [(40 << 20) + 3, 1500, 0, (70 << 20) + 65537, 65536]:
        data = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
        h = BaoHasher()
        assert len(h) == 0
        for off in range(0, total, 3 << 20):
            h.update(data[off:off + (3 << 20)])
        assert len(h) == total
        assert h.finalize() == O.blake3(data)
        assert h.read_all() == O.bao_encode(data)[0]
        del h
        gc.collect()


def test_freed_large_hasher_does_not_keep_its_hbm(gpu):
    """a freed hasher is parked for reuse, but the parked buffers
    are capped (CHIP_HASHER_PARK_MIB, 3 GiB): after hashing 4 GiB (content
    past its first 1 GiB VA range, moved once into a fresh 4x range) and
    freeing the hasher, the device holds at most the cap more than before,
    and drop_cache gives everything back."""
    import gc
    import torch
    from carbonado_amd.utils import BaoHasher
    L = gpu
    L.chip_bao_hasher_drop_cache()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    block = np.random.default_rng(61).integers(0, 256, 256 << 20, dtype=np.uint8)
    h = BaoHasher()
    for _ in range(16):
        h.update(block)
    assert len(h) == 4 << 30
    digest = h.finalize()
    assert digest == O.blake3(block.tobytes() * 16)
    del h
    gc.collect()
    cached = L.chip_bao_hasher_cached_bytes()
    assert cached <= 3 << 30, cached
    held = free0 - torch.cuda.mem_get_info()[0]
    assert held <= (3 << 30) + (256 << 20), held
    L.chip_bao_hasher_drop_cache()
    assert L.chip_bao_hasher_cached_bytes() == 0
    held = free0 - torch.cuda.mem_get_info()[0]
    assert held <= 256 << 20, held


def test_many_live_hashers_then_a_class_balanced_buffer(gpu):
    """every hasher reserves VA for in-place growth and a released
    range is retired (never mapped twice).  Three rounds of 100 hashers alive
    at once (300 in all, 4 parked between rounds) reserve about 1 GiB each
    (was 17 GiB); afterwards chip_device_alloc(1 GiB) still takes the
    class-balanced path, and every digest is exact."""
    import gc
    from carbonado_amd.utils import BaoHasher
    L = gpu
    data = np.random.default_rng(67).integers(0, 256, 100_003, dtype=np.uint8)
    want = O.blake3(data.tobytes())
    for _ in range(3):
        hs = [BaoHasher() for _ in range(100)]
        for h in hs:
            h.update(data)
        assert all(h.finalize() == want for h in hs)
        del hs
        gc.collect()
    L.chip_bao_hasher_drop_cache()
    import ctypes
    p = ctypes.c_void_p()
    assert L.chip_device_alloc(1 << 30, ctypes.byref(p)) == 0
    try:
        f, u, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_double()
        assert L.chip_device_alloc_info(p, ctypes.byref(f), ctypes.byref(u), ctypes.byref(s)) == 0
        assert f.value >= 1 and u.value >= 1
    finally:
        assert L.chip_device_free(p) == 0
