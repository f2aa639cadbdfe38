"""The flat-file container (reference src/file.rs) on the CPU: BIP-340
signatures against the published vectors and the independent Python
restatement (oracle/host_oracle.py), the 160-byte header bytes and parser,
and file::encode / file::decode at the levels without device stages (0-3).
The device levels are in tests/test_gpu_file.py."""
import json

import numpy as np
import pytest

from oracle import host_oracle as H
from oracle import oracle as O

GOLDEN = __import__("pathlib").Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def ca():
    O.build()
    import carbonado_amd
    return carbonado_amd


@pytest.fixture(scope="module")
def vectors():
    return json.loads((GOLDEN / "host_kat.json").read_text())["bip340_sign"]["vectors"]


def _sign(L, sk, msg, aux):
    out = np.zeros(64, np.uint8)
    rc = L.chip_schnorr_sign(sk, len(sk), msg, aux, out.ctypes.data)
    return rc, out.tobytes()


def test_bip340_published_vectors(ca, vectors):
    from carbonado_amd import _lib
    L = _lib.lib()
    for v in vectors:
        sk, pk, aux, msg, sig = (bytes.fromhex(v[k]) for k in ("secret_key", "public_key", "aux_rand", "message",
                                                                  "signature"))
        rc, got = _sign(L, sk, msg, aux)
        assert rc == 0 and got == sig, v["index"]
        assert H.schnorr_sign(sk, msg, aux) == sig  # the oracle is pinned by the same vectors
        assert L.chip_schnorr_verify(pk, 32, msg, sig) == 0
        assert H.schnorr_verify(pk, msg, sig)
        bad = bytearray(sig)
        bad[5] ^= 1
        assert L.chip_schnorr_verify(pk, 32, msg, bytes(bad)) == 18
        assert not H.schnorr_verify(pk, msg, bytes(bad))


def test_sign_verify_matches_oracle_random(ca):
    from carbonado_amd import _lib
    L = _lib.lib()
    for i in range(6):
        sk = H.sha256(b"sk%d" % i)
        msg = H.sha256(b"msg%d" % i)
        aux = H.sha256(b"aux%d" % i)
        rc, sig = _sign(L, sk, msg, aux)
        assert rc == 0 and sig == H.schnorr_sign(sk, msg, aux)
        pub65 = H.public_key(sk)
        pub33 = H.ser_compressed(H.parse_pubkey(pub65))
        for pk in (pub65, pub33, pub33[1:]):
            assert L.chip_schnorr_verify(pk, len(pk), msg, sig) == 0
        assert L.chip_schnorr_verify(pub33, 33, H.sha256(b"other"), sig) == 18
    # fresh auxiliary randomness (the reference's thread_rng): still verifies
    rc, sig = _sign(L, H.sha256(b"k"), H.sha256(b"m"), None)
    assert rc == 0 and H.schnorr_verify(H.ser_compressed(H.parse_pubkey(H.public_key(H.sha256(b"k"))))[1:],
                                        H.sha256(b"m"), sig)
    assert _sign(L, bytes(32), H.sha256(b"m"), None)[0] == 18  # secret key 0


def test_header_bytes_and_parse(ca):
    from carbonado_amd.error import InvalidHeaderLength, InvalidMagicNumber, Secp256k1Error
    from carbonado_amd.file import Header
    sk = H.sha256(b"header sk")
    pk = H.public_key(sk)
    h32 = H.sha256(b"a bao hash")
    aux = H.sha256(b"header aux")
    for meta in (None, b"\x01\x02\x03\x04\x05\x06\x07\x08"):
        hdr = Header.new(sk, pk, h32, 15, 0, 35_660_232, 1941, meta, aux_rand=aux)
        b = hdr.try_to_vec()
        assert len(b) == 160 == Header.len()
        assert b == H.header_bytes(sk, pk, h32, 15, 0, 35_660_232, 1941, meta, aux)
        assert b[:12] == b"CARBONADO01\n" and b[-1] == 0
        back = Header.try_from(b)
        assert back == hdr and back.metadata == meta
        assert H.header_parse(b)["encoded_len"] == 35_660_232
        assert hdr.file_name() == h32.hex() + ".c15"
    b = Header.new(sk, pk, h32, 12, 3, 100, 7, None, aux_rand=aux).try_to_vec()
    with pytest.raises(InvalidHeaderLength):  # the reference panics on a short slice (file.rs:126)
        Header.try_from(b[:158])
    assert Header.try_from(b[:159]).chunk_index == 3  # parse_bytes reads 159 bytes
    with pytest.raises(InvalidMagicNumber):
        Header.try_from(b"X" + b[1:])
    for off in (20, 50, 90, 130):  # pubkey, hash, signature (R), signature (s)
        bad = bytearray(b)
        bad[off] ^= 0x01
        with pytest.raises((Secp256k1Error, ValueError)):
            Header.try_from(bytes(bad))
        with pytest.raises(ValueError):
            H.header_parse(bytes(bad))
    # the format, chunk index and lengths are not signed: they parse as written
    bad = bytearray(b)
    bad[141] = 8
    assert Header.try_from(bytes(bad)).format == 8
    with pytest.raises(Secp256k1Error):  # Message::from_digest_slice: 32 bytes
        Header.new(sk, pk, h32[:31], 12, 0, 0, 0, None)
    with pytest.raises(Secp256k1Error):  # a pubkey that is not a point
        Header.new(sk, b"\x02" + bytes(32), h32, 12, 0, 0, 0, None)


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_file_encode_decode_host_levels(ca, level):
    """file::encode / file::decode at the levels whose stages all run on the
    host; bytes against the oracle (header + restated encode())."""
    from carbonado_amd import file
    sk = H.sha256(b"file sk")
    eph, nonce, aux = H.sha256(b"file eph"), H.sha256(b"file nonce")[:16], H.sha256(b"file aux")
    data = (GOLDEN / "samples" / "contract.rgbc").read_bytes()
    out, info = file.encode(sk, None, data, level, None, ephemeral_sk=eph, nonce=nonce, aux_rand=aux)
    pub33 = H.ser_compressed(H.parse_pubkey(H.public_key(sk)))
    body, h, oinfo = O.c_encode_full(data, level, pub33, eph, nonce)
    assert out == H.header_bytes(sk, pub33, h, level, 0, oinfo["output_len"], oinfo["padding_len"], None, aux) + body
    assert info.output_len == oinfo["output_len"]
    hdr, back = file.decode(sk, out)
    assert back == data and hdr.format == level and hdr.hash == h and hdr.pubkey == pub33


def test_file_encode_given_pubkey_and_metadata(ca):
    from carbonado_amd import file
    from carbonado_amd.error import Secp256k1Error
    sk = H.sha256(b"signer")
    pk = H.public_key(sk)  # 65-byte key: stored compressed
    out, _ = file.encode(sk, pk, b"Hello world!", 3, b"metadata")  # fresh ECIES and signature randomness
    hdr, back = file.decode(sk, out)
    assert back == b"Hello world!" and hdr.metadata == b"metadata"
    assert hdr.pubkey == H.ser_compressed(H.parse_pubkey(pk))
    # file::encode signs with sk but stores the pubkey it is given (file.rs:425-434):
    # with another party's key the file is written, and its header then fails
    # verification on parse, exactly as the reference's would
    other_sk = H.sha256(b"receiver")
    out, _ = file.encode(sk, H.public_key(other_sk), b"Hello world!", 3)
    with pytest.raises(Secp256k1Error):
        file.decode(other_sk, out)


def _fake_device(fail_at=None):
    """Stand-in for device.encode_host_batch (no GPU here): copies each input
    into its output row; raises on slice number `fail_at`."""
    from carbonado_amd.structs import EncodeInfo
    calls = []

    def f(level, inp, n, out, hashes, nslots, pubkey=b"", host_threads=0):
        calls.append(inp.shape[0])
        if fail_at is not None and len(calls) - 1 == fail_at:
            raise RuntimeError("device stage failed")
        cnt = inp.shape[0]
        out[:, :n] = inp[:, :n]
        hashes.zero_()
        hashes[:, 0] = len(calls)
        hashes[:, 1] = __import__("torch").arange(cnt, dtype=__import__("torch").uint8)
        infos = [EncodeInfo(n, n, 0, 0.0, 0, 0, 0, 0.0, 0, 0, 0, 0) for _ in range(cnt)]
        return [n] * cnt, infos
    return f, calls


def _files(tmp_path, count, n=4096):
    d = tmp_path / "in"
    d.mkdir()
    paths = []
    for i in range(count):
        p = d / f"f{i}"
        p.write_bytes(bytes([i & 255]) * n)
        paths.append(p)
    return paths


def test_encode_files_pipeline_ok(ca, tmp_path, monkeypatch):
    """encode_files' three stages end to end with a stand-in device stage."""
    from carbonado_amd import device, file
    f, calls = _fake_device()
    monkeypatch.setattr(device, "encode_host_batch", f)
    paths = _files(tmp_path, 7)
    out = tmp_path / "out"
    out.mkdir()
    sk = H.sha256(b"writer")
    res = file.encode_files(paths, out, sk, 12, slice_objects=2, io_threads=2)
    assert calls == [2, 2, 2, 1]
    assert len(res) == 7 and all(r is not None for r in res)
    for i, (p, info) in enumerate(res):
        body = p.read_bytes()
        assert body[file.HEADER_LEN:] == bytes([i & 255]) * 4096


@pytest.mark.timeout(60)
def test_encode_files_writer_error_raises(ca, tmp_path, monkeypatch):
    """A failing write stage (out_dir is a file) with 3+ slices raises instead
    of hanging (the writer never returned its buffers)."""
    from carbonado_amd import device, file
    f, _ = _fake_device()
    monkeypatch.setattr(device, "encode_host_batch", f)
    paths = _files(tmp_path, 9)
    not_a_dir = tmp_path / "plainfile"
    not_a_dir.write_bytes(b"x")
    with pytest.raises(OSError):
        file.encode_files(paths, not_a_dir, H.sha256(b"w"), 12, slice_objects=2, io_threads=2)


@pytest.mark.timeout(60)
@pytest.mark.parametrize("fail_at", [0, 2])
def test_encode_files_device_error_raises(ca, tmp_path, monkeypatch, fail_at):
    """A device stage that raises (first or a later slice) propagates, with
    the reader and writer threads released (the reader blocked on a
    buffer the main loop never returned)."""
    from carbonado_amd import device, file
    f, _ = _fake_device(fail_at)
    monkeypatch.setattr(device, "encode_host_batch", f)
    paths = _files(tmp_path, 9)
    out = tmp_path / "out"
    out.mkdir()
    with pytest.raises(RuntimeError, match="device stage failed"):
        file.encode_files(paths, out, H.sha256(b"w"), 12, slice_objects=2, io_threads=2)


@pytest.mark.timeout(60)
def test_encode_files_reader_error_raises(ca, tmp_path, monkeypatch):
    """A short read (a file shrinks after the size check) raises."""
    from carbonado_amd import device, file
    f, _ = _fake_device()
    monkeypatch.setattr(device, "encode_host_batch", f)
    paths = _files(tmp_path, 9)
    import pathlib
    orig = pathlib.Path.stat
    out = tmp_path / "out"
    out.mkdir()
    paths[5].write_bytes(b"")
    monkeypatch.setattr(pathlib.Path, "stat", lambda self, *a, **k: orig(paths[0]) if self == paths[5] else orig(self, *a, **k))
    with pytest.raises(IOError):
        file.encode_files(paths, out, H.sha256(b"w"), 12, slice_objects=2, io_threads=2)


def test_sign_scalar_edge_cases_match_oracle(ca):
    """The constant-time scalar arithmetic mod n (secp256k1_host.hpp sc_*):
    keys and messages at the edges of the reductions (d = 1, 2, n - 1, n - 2,
    2^255, all-ones-ish limbs) and random ones, signatures equal to the
    independent Python restatement's."""
    from carbonado_amd import _lib
    L = _lib.lib()
    n = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    keys = [1, 2, 3, n - 1, n - 2, 1 << 255, (1 << 255) - 1, n >> 1, (n >> 1) + 1,
            0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFE00000000000000000000000000000000]
    keys += [int.from_bytes(H.sha256(b"edge%d" % i), "big") % (n - 1) + 1 for i in range(20)]
    msgs = [bytes(32), b"\xff" * 32, H.sha256(b"m")]
    for i, d in enumerate(keys):
        sk = d.to_bytes(32, "big")
        msg = msgs[i % 3]
        aux = H.sha256(b"aux-edge%d" % i) if i % 2 else b"\xff" * 32
        rc, sig = _sign(L, sk, msg, aux)
        assert rc == 0 and sig == H.schnorr_sign(sk, msg, aux), i
    assert _sign(L, n.to_bytes(32, "big"), msgs[0], bytes(32))[0] == 18  # d = n: not a key
