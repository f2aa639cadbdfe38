"""GPU: every entry point that fills a caller buffer writes every byte below
the length it reports.

The Rust shim's `Vec::with_capacity` + `set_len` (carbonado-hip/src/lib.rs
`into_vec`, `zfec_encode`) and the Python wrappers' uninitialised output
`bytes` (carbonado_amd/_buf.py OutBytes) both rely on it: a byte the library
skipped would surface as stale memory.  Each call runs twice, into buffers
pre-filled with 0xA5 and with 0x5A; the reported lengths and every byte below
them must agree (a skipped byte keeps its fill and differs).  Reference
entry points: encoding.rs:38-81, decoding.rs:21-212, utils.rs:104-137,
file.rs:395-440."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 1000, 4096 + 3, 70_000 + 13, (1 << 20) + 5]
SK = bytes(range(1, 33))
EPH = bytes(range(101, 133))
NONCE = bytes(range(7, 23))


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), np.uint8) if len(b) else np.zeros(1, np.uint8)


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _rnd(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _twice(cap: int, call, fixed_len: int | None = None) -> bytes:
    """Run call(out_ptr, cap, len_ref) into 0xA5- and 0x5A-filled buffers;
    assert status 0, equal lengths, and equal bytes below the length."""
    outs = []
    for fill in (0xA5, 0x5A):
        buf = np.full(max(cap, 1) + 64, fill, np.uint8)  # 64 guard bytes past cap
        olen = ctypes.c_uint64(0)
        rc = call(_p(buf), cap, ctypes.byref(olen))
        assert rc == 0, rc
        n = fixed_len if fixed_len is not None else olen.value
        assert n <= cap
        assert (buf[cap:] == fill).all(), "wrote past out_cap"
        outs.append(buf[:n].tobytes())
    assert outs[0] == outs[1], "a byte below the reported length kept its fill"
    return outs[0]


def _inject():
    from carbonado_amd import _lib
    e, n = _u8(EPH), _u8(NONCE)
    return _lib.EciesInjectC(e.ctypes.data, n.ctypes.data), (e, n)


@pytest.mark.parametrize("n", SIZES)
def test_zfec_encode_writes_every_byte(gpu, n):
    L = gpu
    d = _u8(_rnd(n, n))
    total = L.chip_zfec_encoded_len(n, 4, 8)
    pad, chunk = ctypes.c_uint32(), ctypes.c_uint32()
    _twice(total, lambda o, c, ln: L.chip_zfec_encode(4, 8, _p(d), n, o, c, ctypes.byref(pad), ctypes.byref(chunk)),
           fixed_len=total)


@pytest.mark.parametrize("n", SIZES)
def test_stage_functions_write_every_byte(gpu, n):
    import carbonado_amd as ca
    L = gpu
    raw = _rnd(n, n + 1)
    d = _u8(raw)
    # encoding::bao / decoding::bao
    h = np.zeros(32, np.uint8)
    enc = _twice(L.chip_bao_encoded_len(n), lambda o, c, ln: L.chip_bao_encode(_p(d), n, o, c, ln, _p(h)))
    e = _u8(enc)
    assert _twice(n, lambda o, c, ln: L.chip_bao_decode(_p(e), len(enc), _p(h), 32, o, c, ln)) == raw
    # decoding::zfec (positional) and zfec_chunks with explicit indices (two data shards lost)
    shards, pad, chunk = ca.encoding.zfec(raw)
    s = _u8(shards)
    assert _twice(4 * chunk, lambda o, c, ln: L.chip_zfec_decode(4, 8, _p(s), len(shards), pad, o, c, ln)) == raw
    keep = [0, 3, 4, 5, 6, 7]
    rows = [_u8(shards[i * chunk:(i + 1) * chunk]) for i in keep]
    ptrs = (ctypes.c_void_p * len(keep))(*[r.ctypes.data for r in rows])
    idx = (ctypes.c_uint32 * len(keep))(*keep)
    assert _twice(4 * chunk, lambda o, c, ln: L.chip_zfec_decode_shares(4, 8, ptrs, idx, len(keep), chunk, pad, o,
                                                                        c, ln)) == raw


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("level", [4, 8, 12, 15])
def test_encode_decode_write_every_byte(gpu, n, level):
    from carbonado_amd import _lib
    from carbonado_amd.encoding import public_key
    L = gpu
    raw = _rnd(n, 3 * n + level)
    d = _u8(raw)
    pk = _u8(public_key(SK))
    inj, keep = _inject()
    h = np.zeros(32, np.uint8)
    info = _lib.EncodeInfoC()
    enc = _twice(L.chip_encode_max_len(n), lambda o, c, ln: L.chip_encode(
        level, _p(pk), pk.size if level & 1 else 0, ctypes.byref(inj), _p(d), n, o, c, ln, _p(h),
        ctypes.byref(info)))
    e, sk = _u8(enc), _u8(SK)
    back = _twice(n + 1024, lambda o, c, ln: L.chip_decode(_p(sk), 32, _p(h), 32, _p(e), len(enc),
                                                           info.padding_len, level, o, c, ln))
    assert back == raw


@pytest.mark.parametrize("n", [1000, 70_000 + 13, (1 << 20) + 5])
@pytest.mark.parametrize("level", [5, 6, 7, 13, 14, 15])
@pytest.mark.parametrize("where", ["node", "content"])
def test_failed_verdict_leaves_no_plaintext(gpu, n, level, where):
    """decode() at a level with host stages runs them on the content while
    the device verifies; a failed verdict returns BaoDecodeError(HashMismatch)
    (decoding.rs:89-93) and the caller's buffer holds no decoded byte:
    every byte is the fill or wiped.  A damaged parent node (content intact,
    so the host stages succeed) and a damaged content byte."""
    from carbonado_amd import _lib
    from carbonado_amd.encoding import public_key
    L = gpu
    raw = np.frombuffer(_rnd(n, n + level), np.uint8).copy()
    raw[::3] = 0x41  # compressible: the snappy stage decodes real blocks
    raw = raw.tobytes()
    d = _u8(raw)
    pk = _u8(public_key(SK))
    inj, keep = _inject()
    h = np.zeros(32, np.uint8)
    info = _lib.EncodeInfoC()
    enc = bytearray(_twice(L.chip_encode_max_len(n), lambda o, c, ln: L.chip_encode(
        level, _p(pk), pk.size if level & 1 else 0, ctypes.byref(inj), _p(d), n, o, c, ln, _p(h),
        ctypes.byref(info))))
    if where == "node" and len(enc) > 8 + 1024 + 64:
        enc[8 + 5] ^= 0x10  # the root's left child hash (pre-order: the first parent node)
    else:
        enc[len(enc) // 2] ^= 0x10
    e, sk = _u8(enc), _u8(SK)
    cap = n + 1024
    buf = np.full(cap + 64, 0xA5, np.uint8)
    olen = ctypes.c_uint64(7)
    rc = L.chip_decode(_p(sk), 32, _p(h), 32, _p(e), len(enc), info.padding_len, level, _p(buf), cap,
                       ctypes.byref(olen))
    assert rc == 5, rc  # CHIP_ERR_BAO_HASH_MISMATCH
    assert olen.value == 7
    assert np.isin(buf, [0, 0xA5]).all(), "decoded bytes left behind after a failed verdict"


def test_host_stages_write_every_byte(gpu):
    from carbonado_amd.encoding import public_key
    L = gpu
    raw = _rnd(300_000, 9) + bytes(200_000)  # compressible tail: snappy's compressed chunks too
    d = _u8(raw)
    comp = _twice(L.chip_snap_max_len(d.size), lambda o, c, ln: L.chip_snap_compress(_p(d), d.size, o, c, ln))
    cd = _u8(comp)
    assert _twice(d.size, lambda o, c, ln: L.chip_snap_decompress(_p(cd), cd.size, o, c, ln)) == raw
    pk = _u8(public_key(SK))
    inj, keep = _inject()
    ct = _twice(d.size + 97, lambda o, c, ln: L.chip_ecies_encrypt(_p(pk), pk.size, ctypes.byref(inj), _p(d), d.size,
                                                                   o, c, ln))
    ctu, sk = _u8(ct), _u8(SK)
    assert _twice(d.size, lambda o, c, ln: L.chip_ecies_decrypt(_p(sk), 32, _p(ctu), ctu.size, o, c, ln)) == raw


@pytest.mark.parametrize("n", [70_000 + 13, (1 << 20) + 5])
def test_slices_and_scrub_write_every_byte(gpu, n):
    import carbonado_amd as ca
    L = gpu
    raw = _rnd(n, n + 7)
    enc, h, info = ca.encode(b"", raw, 12)
    e, hh = _u8(enc), _u8(h)
    ln_all = len(enc)
    _twice(ln_all, lambda o, c, ln: L.chip_bao_extract_slice(_p(e), ln_all, 3, 1024, o, c, ln))
    spc = info.chunk_slice_count
    _twice(ln_all, lambda o, c, ln: L.chip_bao_verify_slice(_p(hh), 32, _p(e), ln_all, spc, spc, o, c, ln))
    bad = bytearray(enc)
    chunk = ca.extract_slice(enc, 1, 1)[-1024:]
    bad[enc.index(chunk) + 5] ^= 1
    b = _u8(bad)
    assert _twice(ln_all, lambda o, c, ln: L.chip_scrub(_p(b), ln_all, _p(hh), 32, info.padding_len,
                                                        info.chunk_len, o, c, ln)) == enc


def test_hasher_read_all_writes_every_byte(gpu):
    from oracle import oracle as O
    L = gpu
    raw = _rnd((5 << 20) + 77, 11)
    d = _u8(raw)
    h = ctypes.c_void_p()
    assert L.chip_bao_hasher_new(ctypes.byref(h)) == 0
    try:
        for off in range(0, d.size, 1 << 20):
            part = d[off:off + (1 << 20)]
            assert L.chip_bao_hasher_update(h, _p(part), part.size) == 0
        dig = np.zeros(32, np.uint8)
        assert L.chip_bao_hasher_finalize(h, _p(dig)) == 0
        enc = _twice(L.chip_bao_encoded_len(d.size), lambda o, c, ln: L.chip_bao_hasher_read_all(h, o, c, ln))
    finally:
        L.chip_bao_hasher_free(h)
    assert enc == O.bao_encode(raw)[0]


@pytest.mark.parametrize("level", [12, 15])
def test_file_container_writes_every_byte(gpu, level):
    from carbonado_amd import _lib
    from carbonado_amd.encoding import public_key
    L = gpu
    raw = _rnd(200_003, level)
    d, sk, pk = _u8(raw), _u8(SK), _u8(public_key(SK))
    inj, keep = _inject()
    aux = _u8(bytes(32))
    info = _lib.EncodeInfoC()
    cap = 160 + L.chip_encode_max_len(d.size)
    f = _twice(cap, lambda o, c, ln: L.chip_file_encode(_p(sk), 32, _p(pk), pk.size, _p(d), d.size, level, None,
                                                        ctypes.byref(inj), _p(aux), o, c, ln, ctypes.byref(info)))
    fu = _u8(f)
    hdr = _lib.HeaderC()
    assert _twice(d.size + 1024, lambda o, c, ln: L.chip_file_decode(_p(sk), 32, _p(fu), fu.size, ctypes.byref(hdr),
                                                                     o, c, ln)) == raw
