"""bao slice extraction (decoding.rs:116-127) vs the independent Python
restatement of bao's slice rules.  chip_bao_extract_slice is byte selection
along the tree (no arithmetic on the data), so it runs without a device."""
import random

import pytest

from carbonado_amd import decoding
from oracle import oracle as O
from oracle import pyoracle as P


@pytest.mark.parametrize("n", [0, 1, 1024, 1025, 3000, 8192, 8193, 20 * 1024 + 5])
def test_extract_slice_matches_oracle(n):
    d = random.Random(n).randbytes(n)
    enc, h = O.bao_encode(d)
    chunks = max(1, -(-n // 1024))
    for index in sorted({0, 1, chunks // 2, chunks - 1, chunks, chunks + 3}):
        for slen in (0, 1, 1024, 1500, 4096):
            got = decoding.extract_slice(enc, index, slen)
            assert got == P.bao_slice(enc, index * 1024, slen), (n, index, slen)


def test_slice_len_helper():
    from carbonado_amd import _lib
    d = random.Random(9).randbytes(50_000)
    enc, _ = O.bao_encode(d)
    for start, slen in [(0, 1024), (7 * 1024, 3000), (60_000, 10)]:
        assert _lib.lib().chip_bao_slice_len(len(d), start, slen) == len(P.bao_slice(enc, start, slen))


def test_extract_whole_stream_is_the_encoding():
    d = random.Random(1).randbytes(9000)
    enc, _ = O.bao_encode(d)
    assert decoding.extract_slice(enc, 0, len(d)) == enc
