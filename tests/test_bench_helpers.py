"""CPU tests of bench.py's host-side helpers (no device)."""
import sys
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


@pytest.mark.parametrize("n", [4096 * 3, 70_001, 1 << 20, (1 << 20) + 37])
def test_scrub_corrupt_offset_lands_in_a_chunk(n):
    """--mode scrub flips one byte per object at scrub_corrupt_offset(n, o): a
    content byte of data shard o % 4 in the level-12 stream (the layout
    formula 8 + 1024 i + 64 (P(i) + c(i)), checked against the oracle's
    encode)."""
    import bench
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, _, _ = O.encode(d, 12)
    z, _, C = O.zfec_encode(d)
    for o in range(4):
        off = bench.scrub_corrupt_offset(n, o)
        i = o * (C // 1024) + (C // 1024) // 3  # the chunk the helper aims at
        assert enc[off - 517:off - 517 + 1024] == z[1024 * i:1024 * (i + 1)]
