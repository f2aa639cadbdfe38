"""CPU tests of the C-ABI boundary (no compute calls need a GPU here).

* libcarbonado_hip.so loads and exports exactly the symbols
  include/carbonado_hip.h declares, with the ctypes table in _lib.py in sync;
* the host-only size helpers agree with the oracle;
* without a gfx950 device every compute entry point fails loudly
  (CHIP_ERR_NO_DEVICE) — there is no CPU fallback.
"""
import re
import subprocess

import numpy as np
import pytest

from carbonado_amd import _lib
from oracle import oracle as O

HEADER = _lib.LIB_PATH.parents[2] / "include" / "carbonado_hip.h"


def header_symbols() -> set:
    text = HEADER.read_text()
    return set(re.findall(r"^CHIP_API\s+[\w\s\*]+?\b(chip_\w+)\s*\(", text, flags=re.M))


def test_library_built():
    assert _lib.LIB_PATH.exists(), "run __graft_entry__.build()"


def test_exports_match_header():
    syms = header_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert syms == {s for s in exported if s.startswith("chip_")}
    assert syms == set(_lib.SIGNATURES)


def test_library_loads_and_binds_every_symbol():
    L = _lib.lib()
    for name in header_symbols():
        assert getattr(L, name) is not None
    assert L.chip_abi_version() == 5
    assert L.chip_strerror(3).decode().startswith("Input bytes must divide evenly")


@pytest.mark.parametrize("n", [0, 1, 1243, 4096, 4097, 616565, 10240, 16 << 20, (16 << 20) + 2155])
def test_size_helpers_match_oracle(n):
    from carbonado_amd.utils import calc_padding_len
    assert calc_padding_len(n) == O.calc_padding_len(n)
    assert calc_padding_len(n, 8) == O.calc_padding_len(n, 8)
    L = _lib.lib()
    pad, C = O.calc_padding_len(n)
    assert L.chip_zfec_encoded_len(n, 4, 8) == 8 * C
    assert L.chip_bao_encoded_len(n) == O.lib().orc_bao_encoded_len(n)
    assert L.chip_encode_max_len(n) >= O.lib().orc_encode_max_len(n) - 0


def test_bao_scratch_len():
    L = _lib.lib()
    N0 = (32 << 10) // 2  # level-1 nodes (CPL = 2 chunks per lane)
    assert L.chip_bao_scratch_len(32 << 20, 2) == 2 * 32 * (N0 + N0 // 2)


def _has_gfx950() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gfx950(), reason="checks the no-device behaviour")
def test_no_device_fails_loudly():
    import carbonado_amd
    from carbonado_amd.error import DeviceError
    L = _lib.lib()
    assert L.chip_init(0) == 100
    with pytest.raises(DeviceError):
        carbonado_amd.encoding.zfec(b"hello world")
    with pytest.raises(DeviceError):
        carbonado_amd.encode(b"", b"hello", 12)
    with pytest.raises(DeviceError):
        carbonado_amd.encoding.blake3(b"abc")


def test_argument_errors_before_device():
    """Reference error variants that are decided before any compute."""
    import carbonado_amd
    from carbonado_amd import error as E
    with pytest.raises(E.InvalidArgument):
        carbonado_amd.encode(b"", b"x", 15)  # the Ecies bit needs a receiver key
    with pytest.raises(E.EciesError):
        carbonado_amd.encoding.ecies(b"\x04" + b"\0" * 64, b"x")  # not a curve point
    with pytest.raises(E.EciesError):
        carbonado_amd.decoding.ecies(b"\0" * 96, b"\1" * 32)  # shorter than the 97-byte envelope
    with pytest.raises(E.SnapError):
        carbonado_amd.decoding.snap(b"\x01\x05\x00\x00abcde")  # no stream identifier
    with pytest.raises(E.HashDecodeError):
        carbonado_amd.decoding.bao(b"\0" * 8, b"\0" * 31)  # utils.rs:38-45
    with pytest.raises(E.UnevenZfecChunks):
        carbonado_amd.decoding.zfec(np.zeros(1001, np.uint8), 0)  # decoding.rs:39-41


def test_encode_info_fields_match_c_struct():
    """device.encode_host_batch builds EncodeInfo(*row) from the C struct's
    field tuples: the dataclass must list the fields in the struct's order."""
    import dataclasses
    from carbonado_amd import _lib
    from carbonado_amd.structs import EncodeInfo
    assert [f.name for f in dataclasses.fields(EncodeInfo)] == [n for n, _ in _lib.EncodeInfoC._fields_]
