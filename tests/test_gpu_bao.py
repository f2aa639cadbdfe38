"""GPU parity: BLAKE3 / bao kernels (K3/K4/K5) vs the CPU oracle."""
import json

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# from 64 KiB up, encode runs the content mode (K13 KIND 1) on the whole 64-chunk
# blocks and the tail kernel on the rest: tails of 1 byte, 2 chunks, 9 whole
# chunks, 64 chunks with a short last one
SIZES = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3073, 8192, 8193, 65536, 65536 + 1, 65 * 1024 + 7,
         131072 - 5, 4 * 65536 + 9 * 1024, (1 << 20) + 3, 3 * (1 << 20) + 1024 * 5]


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def test_blake3_published_vectors(gpu, golden_dir):
    from carbonado_amd import encoding
    kat = json.loads((golden_dir / "blake3_kat.json").read_text())
    for s, h in kat["strings"].items():
        assert encoding.blake3(s.encode()).hex() == h
    for n, h in kat["pattern_251"].items():
        assert encoding.blake3(bytes(i % 251 for i in range(int(n)))).hex() == h, n


@pytest.mark.parametrize("n", SIZES)
def test_bao_encode_matches_oracle(gpu, n):
    from carbonado_amd import encoding
    d = rnd(n, n)
    enc, h = encoding.bao(d)
    oe, oh = O.bao_encode(d)
    assert h == oh
    assert enc == oe


@pytest.mark.parametrize("n", SIZES)
def test_bao_decode_roundtrip(gpu, n):
    from carbonado_amd import decoding
    d = rnd(n, n + 1)
    enc, h = O.bao_encode(d)
    assert decoding.bao(enc, h) == d


def test_bao_decode_rejects_tampering(gpu):
    from carbonado_amd import decoding
    from carbonado_amd.error import BaoDecodeError
    d = rnd(10_000, 9)
    enc, h = O.bao_encode(d)
    # header, root parent, inner parent, first/last chunk bytes
    for pos in [0, 3, 8, 40, 72 + 10, 200, 4000, len(enc) - 1]:
        t = bytearray(enc)
        t[pos] ^= 0x40
        with pytest.raises(BaoDecodeError):
            decoding.bao(bytes(t), h)
    with pytest.raises(BaoDecodeError) as ei:
        decoding.bao(enc[:-1], h)
    assert ei.value.kind == "Truncated"
    bad = bytearray(h)
    bad[0] ^= 1
    with pytest.raises(BaoDecodeError):
        decoding.bao(enc, bytes(bad))


def test_bao_single_chunk_root_mismatch(gpu):
    from carbonado_amd import decoding
    from carbonado_amd.error import BaoDecodeError
    enc, h = O.bao_encode(b"hello world")
    t = bytearray(enc)
    t[9] ^= 1
    with pytest.raises(BaoDecodeError):
        decoding.bao(bytes(t), h)


def test_batch_bao_full_size(gpu):
    """32 MiB streams (the cfg2 zfec output size, N = 32768 chunks) and a
    non-power-of-two chunk count (cfg4's 32776)."""
    import torch
    from carbonado_amd import device
    for n, count in [(32 << 20, 3), (32776 * 1024, 2)]:
        gen = torch.Generator(device="cuda").manual_seed(n % 1000)
        inp = torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=gen)
        blen = O.lib().orc_bao_encoded_len(n)
        out = torch.empty((count, (blen + 15) // 16 * 16), dtype=torch.uint8, device="cuda")
        hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
        scratch = device.bao_scratch(n, count)
        device.bao_encode_batch(inp, n, out, hashes, scratch)
        torch.cuda.synchronize()
        d0 = inp[0].cpu().numpy().tobytes()
        oe, oh = O.bao_encode(d0)
        assert hashes[0].cpu().numpy().tobytes() == oh
        assert out[0, :blen].cpu().numpy().tobytes() == oe
        for o in range(1, count):
            assert hashes[o].cpu().numpy().tobytes() == O.blake3(inp[o].cpu().numpy().tobytes())
        # verify-decode the whole batch, then corrupt one object
        dec = torch.empty((count, n), dtype=torch.uint8, device="cuda")
        status = torch.empty(count, dtype=torch.int32, device="cuda")
        device.bao_decode_batch(out, n, hashes, dec, status, scratch)
        torch.cuda.synchronize()
        assert torch.equal(dec, inp) and int(status.abs().sum()) == 0
        out[count - 1, 12345] ^= 1
        device.bao_decode_batch(out, n, hashes, dec, status, scratch)
        torch.cuda.synchronize()
        st = status.cpu().tolist()
        assert st[:-1] == [0] * (count - 1) and st[-1] == 5


def test_batch_bao_every_line_phase(gpu):
    """Output streams whose bases take every 8-B phase modulo a 128-B line:
    the encode stream path aligns its whole-line stores to memory, so each
    phase takes a different head/line/tail split (bao_device.hpp stream_lines)."""
    import torch
    from carbonado_amd import device
    n, count = 9 * 1024 + 37, 16
    blen = O.lib().orc_bao_encoded_len(n)
    stride = (blen + 15) // 16 * 16 + 8  # 8 mod 16: o * stride mod 128 visits all 16 phases
    gen = torch.Generator(device="cuda").manual_seed(77)
    inp = torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=gen)
    out = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    device.bao_encode_batch(inp, n, out, hashes, device.bao_scratch(n, count))
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    assert {(out.data_ptr() + o * stride) % 128 for o in range(count)} == set(range(0, 128, 8))
    for o in range(count):
        oe, oh = O.bao_encode(inp[o].cpu().numpy().tobytes())
        assert hashes[o].cpu().numpy().tobytes() == oh, o
        assert host[o, :blen].tobytes() == oe, o
        assert (host[o, blen:] == 0xA5).all(), o  # nothing written past the stream


def test_batch_bao_ragged_large(gpu):
    """A 144 MiB batch of 16 MiB + 37 B objects: a short last chunk, an
    8 mod 16 output stride (the line phase of each stream start differs across
    objects) and a ragged input stride; nothing written past a stream."""
    import torch
    from carbonado_amd import device
    n, count = (16 << 20) + 37, 9
    blen = O.lib().orc_bao_encoded_len(n)
    stride = (blen + 15) // 16 * 16 + 8
    gen = torch.Generator(device="cuda").manual_seed(91)
    inp = torch.randint(0, 256, (count, n + 5), dtype=torch.uint8, device="cuda", generator=gen)
    out = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    device.bao_encode_batch(inp, n, out, hashes, device.bao_scratch(n, count))
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for o in range(count):
        oe, oh = O.bao_encode(inp[o, :n].cpu().numpy().tobytes())
        assert hashes[o].cpu().numpy().tobytes() == oh, o
        assert host[o, :blen].tobytes() == oe, o
        assert (host[o, blen:] == 0xA5).all(), o


@pytest.mark.parametrize("n", [65536 + 1, 131072 - 5, 40 * 65536 + 17 * 1024 + 999, (16 << 20) + 37])
def test_batch_bao_content_mode_tail(gpu, n):
    """Content-mode bao encode of sizes 64 KiB does not divide: K13 KIND 1 on
    the whole 64-chunk blocks, the tail kernel on the last < 64 chunks (their
    levels 1-3 and level-3 CVs), the parent kernels from level 4.  Output
    bases at every 8-B phase of a 128-B line, nothing written past a stream."""
    import torch
    from carbonado_amd import device
    count = 16 if n < (1 << 20) else 3
    blen = O.lib().orc_bao_encoded_len(n)
    stride = (blen + 15) // 16 * 16 + 8
    istride = (n + 15) // 16 * 16
    gen = torch.Generator(device="cuda").manual_seed(n % 9973)
    inp = torch.randint(0, 256, (count, istride), dtype=torch.uint8, device="cuda", generator=gen)
    out = torch.full((count, stride), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    device.bao_encode_batch(inp, n, out, hashes, device.bao_scratch(n, count))
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    for o in range(count):
        oe, oh = O.bao_encode(inp[o, :n].cpu().numpy().tobytes())
        assert hashes[o].cpu().numpy().tobytes() == oh, o
        assert host[o, :blen].tobytes() == oe, o
        assert (host[o, blen:] == 0xA5).all(), o


@pytest.mark.parametrize("n", [3000, 200_000])
def test_bao_decode_mismatch_leaves_no_content(gpu, n):
    """chip_bao_decode reads the verdict and copies the content out behind one
    synchronisation; on a mismatch the caller's buffer is wiped, never left
    holding unverified bytes (KS for 3000 B, the batch kernels for 200 KB)."""
    import ctypes
    import numpy as np
    from carbonado_amd import _lib
    L = _lib.lib()
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    enc, h = O.bao_encode(d)
    bad = bytearray(enc)
    bad[-3] ^= 0x20
    bad = np.frombuffer(bytes(bad), np.uint8)
    out = np.full(n, 0xAA, np.uint8)
    hh = np.frombuffer(h, np.uint8)
    olen = ctypes.c_uint64()
    rc = L.chip_bao_decode(bad.ctypes.data, bad.size, hh.ctypes.data, 32, out.ctypes.data, out.size,
                           ctypes.byref(olen))
    assert rc == 5 and not out.any()
    good = np.frombuffer(enc, np.uint8)
    rc = L.chip_bao_decode(good.ctypes.data, good.size, hh.ctypes.data, 32, out.ctypes.data, out.size,
                           ctypes.byref(olen))
    assert rc == 0 and olen.value == n and out.tobytes() == d


@pytest.mark.parametrize("n", [257 * 1024 + 77, 600 * 1024 + 5])
def test_batch_bao_many_small_trees(gpu, n):
    """2048 objects: the top-of-tree walk runs one wave per object
    (bao_tree.hpp bao_top_kernel TPB 64, batches of >= 2048 trees), straight
    from the chunk CVs (258 chunks) or after one K4 level (601 chunks).  Every
    hash vs the oracle, three whole streams, the batch verify-decode, and one
    damaged parent node flagged on its object only."""
    import torch
    from carbonado_amd import device
    count = 2048
    gen = torch.Generator(device="cuda").manual_seed(n % 997)
    inp = torch.randint(0, 256, (count, n), dtype=torch.uint8, device="cuda", generator=gen)
    blen = O.lib().orc_bao_encoded_len(n)
    out = torch.empty((count, (blen + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    scratch = device.bao_scratch(n, count)
    device.bao_encode_batch(inp, n, out, hashes, scratch)
    torch.cuda.synchronize()
    h_in, h_hash = inp.cpu().numpy(), hashes.cpu().numpy()
    for o in range(count):
        assert h_hash[o].tobytes() == O.blake3(h_in[o].tobytes()), o
    for o in (0, 1237, count - 1):
        assert out[o, :blen].cpu().numpy().tobytes() == O.bao_encode(h_in[o].tobytes())[0], o
    dec = torch.empty((count, n), dtype=torch.uint8, device="cuda")
    status = torch.empty(count, dtype=torch.int32, device="cuda")
    device.bao_decode_batch(out, n, hashes, dec, status, scratch)
    torch.cuda.synchronize()
    assert torch.equal(dec, inp) and int(status.abs().sum()) == 0
    out[777, 8 + 3] ^= 1  # the root's left child CV
    device.bao_decode_batch(out, n, hashes, dec, status, scratch)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert st[777] != 0 and int(np.abs(np.delete(st, 777)).sum()) == 0


@pytest.mark.parametrize("n", [65536 + 1, 4 * 65536 + 9 * 1024, 9 * 1024 + 37])
def test_batch_bao_stream_offset(gpu, n):
    """bao streams 56 B into their rows (every chunk and node on a 64-B
    boundary): the content-mode kernel, its tail kernel and K3 write the same
    streams at that phase, nothing before or after them."""
    import torch
    from carbonado_amd import device
    count, off = 5, 56
    gen = torch.Generator(device="cuda").manual_seed(n % 991)
    inp = torch.randint(0, 256, (count, (n + 255) // 256 * 256), dtype=torch.uint8, device="cuda", generator=gen)
    blen = O.lib().orc_bao_encoded_len(n)
    out = torch.full((count, (off + blen + 255) // 256 * 256), 0xA5, dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    device.bao_encode_batch(inp, n, out, hashes, device.bao_scratch(n, count), out_offset=off)
    torch.cuda.synchronize()
    host, h_in = out.cpu().numpy(), inp.cpu().numpy()
    for o in range(count):
        oe, oh = O.bao_encode(h_in[o, :n].tobytes())
        assert hashes[o].cpu().numpy().tobytes() == oh, o
        assert host[o, off:off + blen].tobytes() == oe, o
        assert (host[o, :off] == 0xA5).all() and (host[o, off + blen:] == 0xA5).all(), o
    # the verify-decode reads them at that phase too
    dec = torch.empty((count, (n + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
    status = torch.empty(count, dtype=torch.int32, device="cuda")
    scratch = device.bao_scratch(n, count)
    device.bao_decode_batch(out, n, hashes, dec, status, scratch, in_offset=off)
    torch.cuda.synchronize()
    assert int(status.abs().sum()) == 0 and torch.equal(dec[:, :n], inp[:, :n])
    out[2, off + blen - 1] ^= 1  # the last chunk's last byte
    device.bao_decode_batch(out, n, hashes, dec, status, scratch, in_offset=off)
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    assert st[2] != 0 and st[:2] + st[3:] == [0] * (count - 1)


def _bao_parents(N):
    """(level, offset) of every parent node of an N-chunk bao stream, in
    pre-order (left subtree: the largest power of two below n chunks)."""
    out, pos = [], 8

    def rec(n):
        nonlocal pos
        if n == 1:
            pos += 1024
            return
        left = 1 << ((n - 1).bit_length() - 1)
        out.append(((n - 1).bit_length(), pos))
        pos += 64
        rec(left)
        rec(n - left)
    rec(N)
    return out


@pytest.mark.parametrize("n", [1000 * 1024 + 7, (16 << 20) + 3])
def test_batch_bao_decode_flags_each_parent_level(gpu, n):
    """Verify-decode checks every parent level: one object per level 2 .. 7
    has one byte of one of its level-l nodes flipped (K4 per level, then the
    top walk), each flagged on its own object only; the intact ones decode."""
    import torch
    from carbonado_amd import device
    N = (n + 1023) // 1024
    parents = _bao_parents(N)
    levels = [2, 3, 4, 5, 6, 7]
    count = len(levels) + 2
    gen = torch.Generator(device="cuda").manual_seed(n % 887)
    inp = torch.randint(0, 256, (count, (n + 255) // 256 * 256), dtype=torch.uint8, device="cuda", generator=gen)
    blen = O.lib().orc_bao_encoded_len(n)
    off = 56
    enc = torch.empty((count, (off + blen + 255) // 256 * 256), dtype=torch.uint8, device="cuda")
    hashes = torch.empty((count, 32), dtype=torch.uint8, device="cuda")
    scratch = device.bao_scratch(n, count)
    device.bao_encode_batch(inp, n, enc, hashes, scratch, out_offset=off)
    torch.cuda.synchronize()
    rng = np.random.default_rng(n)
    for o, lv in enumerate(levels, start=1):
        cands = [p for (l, p) in parents if l == lv]
        pos = cands[int(rng.integers(0, len(cands)))] + int(rng.integers(0, 64))
        enc[o, off + pos] ^= 0x10
    dec = torch.empty((count, n), dtype=torch.uint8, device="cuda")
    status = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    device.bao_decode_batch(enc, n, hashes, dec, status, scratch, in_offset=off)
    torch.cuda.synchronize()
    st = status.cpu().tolist()
    assert st[0] == 0 and st[-1] == 0, st
    assert all(x != 0 for x in st[1:-1]), st
    assert torch.equal(dec[0], inp[0, :n]) and torch.equal(dec[-1], inp[-1, :n])
