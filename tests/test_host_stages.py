"""Host stages of encode()/decode(): snappy framing and ECIES.

CPU-only: these stages run on host threads by design (host_stages.cpp; the
reference's encoding.rs:16-36 and decoding.rs:62-77), so the library's
entry points are exercised here without a device, against
  * published known answers (tests/golden/host_kat.json) for the restated
    primitives in oracle/host_oracle.py (SHA-256, HMAC, HKDF, AES-256, GCM,
    CRC-32C, secp256k1), and
  * the oracle itself for the composed stages (byte-exact snap frames and
    ECIES envelopes with injected ephemeral key and nonce), and
  * golden.json's level 1/2/3/14/15 vectors of the reference's sample files.
Parity vs the snap / ecies crates themselves is unpinned (neither builds
here); see DESIGN.md.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import host_oracle as H
from oracle import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def kat():
    return json.loads((GOLDEN / "host_kat.json").read_text())


@pytest.fixture(scope="module")
def golden():
    return json.loads((GOLDEN / "golden.json").read_text())


def _x(h):
    return bytes.fromhex(h)


# ---------------------------------------------------------------- oracle KATs
def test_sha256_hmac_hkdf_kat(kat):
    for v in kat["sha256"]:
        assert H.sha256(_x(v["msg_hex"])).hex() == v["digest"]
    t = kat["hmac_sha256_rfc4231_tc1"]
    assert H.hmac_sha256(_x(t["key_hex"]), _x(t["data_hex"])).hex() == t["mac"]
    for v in kat["hkdf_sha256_rfc5869"]:
        salt = _x(v["salt_hex"]) or None
        assert H.hkdf_sha256(_x(v["ikm_hex"]), salt, _x(v["info_hex"]), v["L"]).hex() == v["okm"]


def test_aes_gcm_kat(kat):
    a = kat["aes256_fips197_c3"]
    assert H.aes256_block(H.aes256_expand(_x(a["key_hex"])), _x(a["pt_hex"])).hex() == a["ct"]
    for v in kat["aes256_gcm"]:
        ct, tag = H.aes256_gcm_encrypt(_x(v["key_hex"]), _x(v["iv_hex"]), _x(v["pt_hex"]))
        assert ct.hex() == v["ct"] and tag.hex() == v["tag"]
        assert H.aes256_gcm_decrypt(_x(v["key_hex"]), _x(v["iv_hex"]), ct, tag) == _x(v["pt_hex"])


def test_crc32c_and_secp256k1_kat(kat):
    assert H.crc32c(kat["crc32c_check"]["msg"].encode()) == int(kat["crc32c_check"]["crc"], 16)
    g = tuple(int(c, 16) for c in kat["secp256k1"]["G"])
    assert H.point_mul(1) == g and H.on_curve(g)
    assert H.point_mul(2) == tuple(int(c, 16) for c in kat["secp256k1"]["2G"])
    assert H.point_mul(H.N) is None  # the generator has order n


def test_oracle_sha256_matches_hashlib():
    import hashlib
    rng = np.random.default_rng(3)
    for n in [0, 1, 55, 56, 63, 64, 65, 127, 1000, 4097]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert H.sha256(d) == hashlib.sha256(d).digest()


def test_oracle_snappy_roundtrip_and_framing(kat):
    rng = np.random.default_rng(4)
    assert H.snap_compress(b"") == _x(kat["snappy_framing"]["empty_input_frame"])
    for d in [b"a", bytes(100), b"abc" * 30000, rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
              rng.integers(0, 3, 140000, dtype=np.uint8).tobytes()]:
        f = H.snap_compress(d)
        assert f.startswith(_x(kat["snappy_framing"]["stream_identifier"]))
        assert H.snap_decompress(f) == d
    # incompressible blocks are stored raw: 10 + n + 8 per 64 KiB block
    r = rng.integers(0, 256, 3 * 65536 + 5, dtype=np.uint8).tobytes()
    assert len(H.snap_compress(r)) == 10 + len(r) + 8 * 4


def test_oracle_golden_host_levels(golden):
    m = golden["ecies_material"]
    sk, eph, nonce = _x(m["secret_key"]), _x(m["ephemeral_sk"]), _x(m["nonce"])
    assert H.public_key(sk).hex() == m["public_key"]
    for name in ["contract.rgbc", "code.tar"]:
        data = (GOLDEN / "samples" / name).read_bytes()
        for level in (1, 2, 3, 14, 15):
            g = golden["samples"][name][f"level{level}"]
            enc, h, info = O.encode_full(data, level, _x(m["public_key"]), eph, nonce)
            assert h.hex() == g["hash"] and len(enc) == g["output_len"]
            assert O.blake3(enc).hex() == g["output_blake3"], (name, level)
            assert O.decode_full(sk, h, enc, info["padding_len"], level) == data


# ---------------------------------------------------------------- product (host code)
@pytest.fixture(scope="module")
def ca():
    import carbonado_amd
    return carbonado_amd


SAMPLES = ["contract.rgbc", "code.tar", "content.png"]


def _inputs():
    rng = np.random.default_rng(9)
    out = [(GOLDEN / "samples" / s).read_bytes() for s in SAMPLES]
    out += [b"", b"x", bytes(17), b"hello world " * 20000, rng.integers(0, 256, 200_003, dtype=np.uint8).tobytes(),
            rng.integers(0, 4, 150_000, dtype=np.uint8).tobytes(), bytes(rng.integers(97, 100, 65536 * 2 + 7))]
    return out


@pytest.mark.parametrize("i", range(10))
def test_snap_compress_matches_oracle(ca, i):
    d = _inputs()[i]
    f = ca.encoding.snap(d)
    assert f == H.snap_compress(d)
    assert ca.decoding.snap(f) == d


def test_snap_decompress_rejects_corruption(ca):
    from carbonado_amd.error import SnapError
    f = bytearray(ca.encoding.snap(b"hello world " * 1000))
    bad = bytearray(f)
    bad[-1] ^= 1  # compressed body / checksum mismatch
    with pytest.raises(SnapError):
        ca.decoding.snap(bytes(bad))
    with pytest.raises(SnapError):
        ca.decoding.snap(bytes(f[:-3]))  # truncated chunk
    with pytest.raises(SnapError):
        ca.decoding.snap(b"\x02\x01\x00\x00x" + bytes(f))  # reserved unskippable chunk first
    # skippable padding chunk after the identifier is ignored
    assert ca.decoding.snap(bytes(f[:10]) + b"\xfe\x02\x00\x00\0\0" + bytes(f[10:])) == b"hello world " * 1000


@pytest.mark.parametrize("keyform", ["uncompressed", "compressed", "raw64"])
def test_ecies_matches_oracle(ca, keyform):
    sk = H.sha256(b"test receiver")
    pub = H.public_key(sk)
    assert ca.encoding.public_key(sk) == pub
    if keyform == "compressed":
        pk = (b"\x02" if H.parse_pubkey(pub)[1] % 2 == 0 else b"\x03") + pub[1:33]
    elif keyform == "raw64":
        pk = pub[1:]
    else:
        pk = pub
    eph, nonce = H.sha256(b"eph"), H.sha256(b"nonce")[:16]
    for d in [b"", b"a", bytes(1000), np.random.default_rng(2).integers(0, 256, 4099, dtype=np.uint8).tobytes()]:
        e = ca.encoding.ecies(pk, d, ephemeral_sk=eph, nonce=nonce)
        assert e == H.ecies_encrypt(pk, d, eph, nonce)
        assert ca.decoding.ecies(e, sk) == d
        assert H.ecies_decrypt(sk, e) == d


@pytest.mark.parametrize("level", [1, 3])
def test_one_pass_encrypt_matches_oracle(ca, level):
    """encode() at Ecies (|Snappy) frames and encrypts block by block through a
    window (host_stages.cpp ecies_encrypt_stream): the same bytes and
    EncodeInfo as snap_compress followed by ecies_encrypt, for empty, tiny,
    compressible, incompressible and multi-block inputs."""
    sk = H.sha256(b"one pass encrypt")
    pub = H.public_key(sk)
    eph, nonce = H.sha256(b"ope"), H.sha256(b"opn")[:16]
    for d in _inputs() + [bytes(np.random.default_rng(5).integers(0, 256, 65536 * 3, dtype=np.uint8))]:
        enc, h, info = ca.encode(pub, d, level, ephemeral_sk=eph, nonce=nonce)
        oenc, oh, oinfo = O.encode_full(d, level, pub, eph, nonce)
        assert enc == oenc, len(d)
        assert info.bytes_compressed == oinfo["bytes_compressed"]
        assert info.bytes_encrypted == oinfo["bytes_encrypted"]
        assert ca.decode(sk, h, enc, info.padding_len, level) == d


def test_ecies_random_envelopes_decrypt(ca):
    """Without injection every call draws a fresh ephemeral key and nonce."""
    sk = H.sha256(b"rng receiver")
    pub = ca.encoding.public_key(sk)
    a, b = ca.encoding.ecies(pub, b"same message"), ca.encoding.ecies(pub, b"same message")
    assert a != b and a[:65] != b[:65] and a[65:81] != b[65:81]
    assert H.ecies_decrypt(sk, a) == b"same message" == ca.decoding.ecies(b, sk)


def test_ecies_errors(ca):
    from carbonado_amd.error import EciesError
    sk = H.sha256(b"err receiver")
    e = ca.encoding.ecies(ca.encoding.public_key(sk), b"payload" * 10)
    for pos in (0 + 40, 70, 90, 100, len(e) - 1):  # eph key, nonce, tag, ciphertext
        bad = bytearray(e)
        bad[pos] ^= 0x40
        with pytest.raises(EciesError):
            ca.decoding.ecies(bytes(bad), sk)
    with pytest.raises(EciesError):
        ca.decoding.ecies(e, H.sha256(b"someone else"))
    with pytest.raises(EciesError):
        ca.decoding.ecies(e, bytes(32))  # zero is not a valid secret key
    with pytest.raises(EciesError):
        ca.decoding.ecies(e, bytes.fromhex("FF" * 32))  # >= group order
    with pytest.raises(EciesError):
        ca.encoding.ecies(b"\x02" + bytes(31), b"x")  # wrong length


def test_ecies_snap_one_pass_decode(ca):
    """decode() with Ecies|Snappy (decoding.rs:101-111) decrypts and unsnaps in
    one pass through a 256 KiB window (host_stages.cpp ecies_decrypt_snap):
    same bytes and error classes as decoding.ecies followed by decoding.snap."""
    from carbonado_amd.error import EciesError, SnapError
    sk = H.sha256(b"one pass receiver")
    pk = ca.encoding.public_key(sk)
    rng = np.random.default_rng(11)
    big = rng.integers(0, 256, 1_000_003, dtype=np.uint8).tobytes()  # raw chunks, 4x the window
    comp = b"carbonado " * 120_000  # compressed chunks; output > decode()'s first guess
    for d in [b"", b"x", big, comp]:
        f = ca.encoding.snap(d)
        e = ca.encoding.ecies(pk, f)
        assert ca.decode(sk, b"", e, 0, 3) == d == ca.decoding.snap(ca.decoding.ecies(e, sk))
        if not f:  # an empty input has an empty stream (no identifier to pad after)
            continue
        # skippable padding chunk larger than the window
        pad = bytes(f[:10]) + b"\xfe" + (300_000).to_bytes(3, "little") + bytes(300_000) + bytes(f[10:])
        assert ca.decode(sk, b"", ca.encoding.ecies(pk, pad), 0, 3) == d
    f = ca.encoding.snap(big)
    bad = bytearray(f)
    bad[-1] ^= 1  # CRC mismatch in the last chunk, valid tag
    with pytest.raises(SnapError):
        ca.decode(sk, b"", ca.encoding.ecies(pk, bytes(bad)), 0, 3)
    with pytest.raises(SnapError):  # truncated frame
        ca.decode(sk, b"", ca.encoding.ecies(pk, bytes(f[:-3])), 0, 3)
    # data chunk longer than the window: the two-pass route, same verdict
    huge = bytes(f[:10]) + b"\x00" + (300_000).to_bytes(3, "little") + bytes(300_000)
    with pytest.raises(SnapError):
        ca.decode(sk, b"", ca.encoding.ecies(pk, huge), 0, 3)
    e = bytearray(ca.encoding.ecies(pk, bytes(bad)))
    e[200] ^= 0x40  # bad tag wins over the snap error
    with pytest.raises(EciesError):
        ca.decode(sk, b"", bytes(e), 0, 3)
    e = bytearray(ca.encoding.ecies(pk, f))
    e[-1] ^= 0x40
    with pytest.raises(EciesError):
        ca.decode(sk, b"", bytes(e), 0, 3)


# ---------------------------------------------------------------- C restatement
def test_c_host_oracle_matches_python_oracle(kat):
    """oracle/host_oracle.c (the full-size checker and CPU baseline) agrees
    with the Python restatement and the published vectors."""
    import ctypes
    L = O.lib()
    assert L.orc_crc32c(b"123456789", 9) == int(kat["crc32c_check"]["crc"], 16)
    out = ctypes.create_string_buffer(32)
    for v in kat["sha256"]:
        m = _x(v["msg_hex"])
        L.orc_sha256(m, len(m), out)
        assert out.raw.hex() == v["digest"]
    t = kat["hmac_sha256_rfc4231_tc1"]
    L.orc_hmac_sha256(_x(t["key_hex"]), 20, _x(t["data_hex"]), 8, out)
    assert out.raw.hex() == t["mac"]
    sk = H.sha256(b"c oracle")
    pub = H.public_key(sk)
    assert O.c_public_key(sk) == pub
    rng = np.random.default_rng(8)
    for d in [b"", b"q", b"carbonado " * 9000, rng.integers(0, 256, 70_001, dtype=np.uint8).tobytes()]:
        f = O.c_snap_compress(d)
        assert f == H.snap_compress(d) and O.c_snap_decompress(f, len(d) + 1) == d
        e = O.c_ecies_encrypt(pub, d[:3000], H.sha256(b"e"), bytes(range(16)))
        assert e == H.ecies_encrypt(pub, d[:3000], H.sha256(b"e"), bytes(range(16)))
        assert O.c_ecies_decrypt(sk, e) == d[:3000]


def test_c_full_pipeline_golden(golden):
    m = golden["ecies_material"]
    for name in SAMPLES:
        data = (GOLDEN / "samples" / name).read_bytes()
        for level in (1, 2, 3, 14, 15):
            enc, h, _ = O.c_encode_full(data, level, _x(m["public_key"]), _x(m["ephemeral_sk"]), _x(m["nonce"]))
            g = golden["samples"][name][f"level{level}"]
            assert O.blake3(enc).hex() == g["output_blake3"] and h.hex() == g["hash"], (name, level)


def _chip_decode_raw(sk, enc, level, out, cap):
    """chip_decode straight through the C-ABI with a caller-owned buffer."""
    import ctypes
    from carbonado_amd import _lib
    L = _lib.lib()
    got = ctypes.c_uint64()
    e = np.frombuffer(enc, np.uint8)
    rc = L.chip_decode(sk, len(sk), None, 0, e.ctypes.data, e.size, 0, level,
                       out.ctypes.data if out is not None else None, cap, ctypes.byref(got))
    return rc, got.value


def test_bad_tag_wipes_written_output(ca):
    """A bad AES-GCM tag returns EciesError and leaves no plaintext in the
    caller's buffer, on the one-pass route and on the two-pass route a data
    chunk longer than the window takes (the fallback used to keep
    the bytes it had already decoded)."""
    sk = H.sha256(b"wipe receiver")
    pk = ca.encoding.public_key(sk)
    rng = np.random.default_rng(21)
    head = rng.integers(0, 256, 500_000, dtype=np.uint8).tobytes()
    f = ca.encoding.snap(head)
    tail = rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes()
    two_pass = bytes(f) + b"\x00" + (300_000).to_bytes(3, "little") + tail  # 300 KB data chunk > 256 KiB window
    for stream in (bytes(f), two_pass):
        e = bytearray(ca.encoding.ecies(pk, stream))
        e[-5] ^= 0x40  # ciphertext of the last chunk: the tag check fails at the end
        out = np.full(2_000_000, 0xAA, np.uint8)
        rc, _ = _chip_decode_raw(sk, bytes(e), 3, out, out.size)
        assert rc == 17  # CHIP_ERR_ECIES
        assert not (out[:len(head)] == np.frombuffer(head, np.uint8)).all()
        assert set(np.unique(out).tolist()) <= {0x00, 0xAA}
        assert (out[:len(head)] == 0).all() or (out[:len(head)] == 0xAA).all()


def test_null_output_sizes_without_writing(ca):
    """out == NULL with a nonzero capacity: BUFFER_TOO_SMALL and the required
    size, nothing written (the one-pass route dereferenced NULL)."""
    sk = H.sha256(b"null receiver")
    pk = ca.encoding.public_key(sk)
    d = b"carbonado " * 5000
    e = ca.encoding.ecies(pk, ca.encoding.snap(d))
    rc, need = _chip_decode_raw(sk, e, 3, None, 1 << 20)
    assert rc == 2 and need == len(d)  # CHIP_ERR_BUFFER_TOO_SMALL


def test_secp256k1_scalar_mult_matches_oracles(ca):
    """The ECIES stage's constant-time secp256k1 (csrc/secp256k1_host.hpp):
    k*G (public_key) and k*P (the ECDH inside encrypt/decrypt) against the
    C oracle's Jacobian code and the Python restatement, for edge scalars and
    random ones."""
    from oracle import oracle as O
    n = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    edge = [1, 2, 3, 15, 16, 17, 255, 256, 2**128, 2**255, n - 1, n - 2, n // 2]
    rng = np.random.default_rng(77)
    rand = [int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "big") % (n - 1) + 1
            for _ in range(60)]
    for k in edge + rand:
        sk = k.to_bytes(32, "big")
        assert ca.encoding.public_key(sk) == O.c_public_key(sk), hex(k)
    for k in edge[:6] + rand[:4]:
        assert ca.encoding.public_key(k.to_bytes(32, "big")) == H.public_key(k.to_bytes(32, "big"))
    # k * P through ECIES: random receivers and ephemeral keys, against the C oracle's envelope
    for i in range(12):
        sk = rand[i].to_bytes(32, "big")
        eph = (edge[i] if i < len(edge) else rand[-i]).to_bytes(32, "big")
        pub = O.c_public_key(sk)
        nonce = bytes(range(16))
        e = ca.encoding.ecies(pub, b"m" * i, ephemeral_sk=eph, nonce=nonce)
        assert e == O.c_ecies_encrypt(pub, b"m" * i, eph, nonce)
        assert ca.decoding.ecies(e, sk) == b"m" * i


@pytest.mark.parametrize("threads", [1, 4])
def test_encode_host_batch_host_levels(ca, threads):
    """chip_encode_host_batch at the host-only levels (Ecies / Snappy, no device
    part) on a team of host threads over several slices (the slice rounded up to
    a multiple of the team): every object equals the oracle's encode()."""
    import torch
    from carbonado_amd import device
    sk = H.sha256(b"team receiver")
    pub = H.public_key(sk)
    n, count = 20_001, 11
    inp = torch.from_numpy(np.random.default_rng(threads).integers(0, 256, (count, n), dtype=np.uint8))
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.zeros((count, cap), dtype=torch.uint8)
    hashes = torch.zeros((count, 32), dtype=torch.uint8)
    eph = np.stack([np.frombuffer(H.sha256(b"te%d" % o), np.uint8) for o in range(count)])
    nonce = np.stack([np.frombuffer(H.sha256(b"tn%d" % o)[:16], np.uint8) for o in range(count)])
    for level in (1, 2, 3):
        olen, _ = device.encode_host_batch(level, inp, n, out, hashes, 3, slice_bytes=3 * n, pubkey=pub,
                                           ephemeral_sk=eph, nonce=nonce, host_threads=threads)
        for o in range(count):
            enc, _, _ = O.encode_full(inp[o].numpy().tobytes(), level, pub, eph[o].tobytes(), nonce[o].tobytes())
            assert out[o, :olen[o]].numpy().tobytes() == enc, (level, o)


def test_encode_host_batch_ecies_key_prep(ca):
    """The batch prepares each object's ECIES key material during its slice's
    slot wait (api_encode.cpp KeyPrep): drawn ephemeral keys still differ per
    object and decrypt with the receiver's secret; a bad receiver key or an
    injected ephemeral secret outside (0, n) fails the call as ecies() does."""
    import torch
    from carbonado_amd import device
    from carbonado_amd.error import EciesError
    sk = H.sha256(b"prep receiver")
    pub = H.public_key(sk)
    n, count = 3000, 9
    inp = torch.from_numpy(np.random.default_rng(5).integers(0, 256, (count, n), dtype=np.uint8))
    cap = device._lib.lib().chip_encode_max_len(n)
    out = torch.zeros((count, cap), dtype=torch.uint8)
    hashes = torch.zeros((count, 32), dtype=torch.uint8)
    olen, _ = device.encode_host_batch(1, inp, n, out, hashes, 2, slice_bytes=4 * n, pubkey=pub, host_threads=3)
    heads = {out[o, :65].numpy().tobytes() for o in range(count)}
    assert len(heads) == count
    for o in range(count):
        assert H.ecies_decrypt(sk, out[o, :olen[o]].numpy().tobytes()) == inp[o].numpy().tobytes()
    with pytest.raises(EciesError):
        device.encode_host_batch(1, inp, n, out, hashes, 2, slice_bytes=4 * n, pubkey=b"\x04" + bytes(64))
    eph = np.stack([np.frombuffer(H.sha256(b"pe%d" % o), np.uint8) for o in range(count)])
    eph[6] = 0  # zero is not a valid secret key
    nonce = np.zeros((count, 16), np.uint8)
    with pytest.raises(EciesError):
        device.encode_host_batch(1, inp, n, out, hashes, 2, slice_bytes=4 * n, pubkey=pub, ephemeral_sk=eph,
                                 nonce=nonce, host_threads=3)


@pytest.mark.parametrize("n", [0, 1, 7, 8, 255, 256, 767, 768, 769, 3 * 256 + 8, 4095, 12287, 12288, 12289,
                               12288 + 767, 3 * 12288 + 5, 65535, 65536, 65537])
def test_snap_frame_crc_lengths(ca, n):
    """The frame CRC-32C of every chunk length class: three crc32q chains over
    segments of 4096 and 256 bytes, joined by table shifts, then one chain for
    the rest (host_stages.cpp crc32c) — frames byte-exact with the oracle's,
    random and compressible data."""
    for data in (np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes(), bytes(n)):
        assert ca.encoding.snap(data) == H.snap_compress(data), n
        assert ca.decoding.snap(ca.encoding.snap(data)) == data


_GCM_LENS = [0, 1, 15, 16, 17, 31, 255, 256, 257, 511, 4095, 4096 + 8, 65536 * 2 + 13, (1 << 20) + 3]


def _gcm_envelopes(ca, seed):
    """ECIES envelopes over _GCM_LENS plus encode() at level 1 (one-pass
    snap+ecies: 8-byte block headers between bodies, so the cipher's update
    splits fall off block boundaries) and their decrypts."""
    sk = H.sha256(b"gcm paths")
    pub = H.public_key(sk)
    eph, nonce = H.sha256(b"gcm eph"), H.sha256(b"gcm nonce")[:16]
    rng = np.random.default_rng(seed)
    out = []
    for n in _GCM_LENS:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        e = ca.encoding.ecies(pub, d, ephemeral_sk=eph, nonce=nonce)
        assert ca.decoding.ecies(e, sk) == d
        out.append(e)
    d = (b"carbonado " * 30_000) + rng.integers(0, 256, 200_001, dtype=np.uint8).tobytes()
    enc, h, info = ca.encode(pub, d, 1, ephemeral_sk=eph, nonce=nonce)
    assert ca.decode(sk, h, enc, info.padding_len, 1) == d
    out.append(enc)
    return out, d


def test_gcm_paths_match_oracle(ca):
    """AES-256-GCM inside ECIES runs on the VAES/VPCLMULQDQ path
    (gcm_vaes.cpp) where the CPU has it and on OpenSSL's EVP otherwise or
    with CHIP_GCM=openssl: both give the C oracle's envelopes byte for byte
    (lengths around the 16-B block and 256-B step, a 1 MiB body, and the
    one-pass encrypt's unaligned update splits), and a flipped tag or
    ciphertext byte is refused on either."""
    import hashlib
    import os
    import subprocess
    import sys
    from carbonado_amd.error import EciesError
    envs, d = _gcm_envelopes(ca, 21)
    sk = H.sha256(b"gcm paths")
    pub = H.public_key(sk)
    eph, nonce = H.sha256(b"gcm eph"), H.sha256(b"gcm nonce")[:16]
    rng = np.random.default_rng(21)
    for n, e in zip(_GCM_LENS, envs):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert e == O.c_ecies_encrypt(pub, m, eph, nonce), n
    oenc, _, _ = O.encode_full(d, 1, pub, eph, nonce)
    assert envs[-1] == oenc
    for pos in (81, 96, 97, len(envs[9]) - 1):  # tag first/last byte, ciphertext first/last
        bad = bytearray(envs[9])
        bad[pos] ^= 1
        with pytest.raises(EciesError):
            ca.decoding.ecies(bytes(bad), sk)
    digest = hashlib.sha256(b"".join(envs)).hexdigest()
    code = ("import hashlib, sys; sys.path.insert(0, 'tests'); import carbonado_amd as ca; "
            "from test_host_stages import _gcm_envelopes; "
            "print(hashlib.sha256(b''.join(_gcm_envelopes(ca, 21)[0])).hexdigest())")
    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, CHIP_GCM="openssl")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == digest


def test_snappy_interop_with_cpp_snappy(ca):
    """An independent pin for the snappy block format: Google's C++ snappy as
    bundled in pyarrow (parity with the snap crate's own compressor stays
    unpinned).  Every compressed chunk of our frames decompresses
    with it to its block, and frames made of its compressed blocks (masked
    CRC-32C from the C oracle) decode with ours; on very compressible blocks
    the two compressors emit the same bytes."""
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("snappy")
    L = O.lib()

    def masked(b):
        c = L.orc_crc32c(b, len(b)) & 0xFFFFFFFF
        return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF

    def chunks(f):
        s, out = 10, []
        while s < len(f):
            ty, cl = f[s], int.from_bytes(f[s + 1:s + 4], "little")
            out.append((ty, f[s + 4:s + 4 + cl]))
            s += 4 + cl
        return out

    rng = np.random.default_rng(31)
    text = b"".join(rng.choice([b"carbonado ", b"archive ", b"zfec ", b"bao "], 40_000).tolist())
    cases = [b"hello world " * 1000, bytes(100_000), text,
             rng.integers(0, 4, 200_000, dtype=np.uint8).tobytes(),
             rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes(),
             (GOLDEN / "samples" / "code.tar").read_bytes(), (GOLDEN / "samples" / "content.png").read_bytes()]
    identical = 0
    for d in cases:
        f = ca.encoding.snap(d)
        o = 0
        for ty, body in chunks(f):
            blk = d[o:o + 65536]
            o += len(blk)
            assert int.from_bytes(body[:4], "little") == masked(blk)
            if ty == 0x00:
                assert codec.decompress(body[4:], decompressed_size=len(blk), asbytes=True) == blk
                identical += body[4:] == codec.compress(blk, asbytes=True)
            else:
                assert ty == 0x01 and body[4:] == blk
        assert o == len(d)
        # the other way: C++ snappy's blocks in a frame, decoded by ours
        frame = bytearray(f[:10])
        for i in range(0, len(d), 65536):
            blk = d[i:i + 65536]
            z = codec.compress(blk, asbytes=True)
            frame += bytes([0x00]) + (4 + len(z)).to_bytes(3, "little") + masked(blk).to_bytes(4, "little") + z
        assert ca.decoding.snap(bytes(frame)) == d
    assert identical >= 8


def _par_inputs():
    rng = np.random.default_rng(41)
    words = [b"carbonado ", b"archive ", b"zfec ", b"bao ", b"segment "]
    text = b"".join(rng.choice(words, 400_000).tolist())
    return [rng.integers(0, 256, 256 * 1024 - 1, dtype=np.uint8).tobytes(),  # one-thread path
            rng.integers(0, 256, 256 * 1024, dtype=np.uint8).tobytes(),      # parallel from here on
            text[:256 * 1024 + 1],
            rng.integers(0, 4, (1 << 20) + 5, dtype=np.uint8).tobytes(),
            text[:3 * (1 << 20) + 17],
            rng.integers(0, 256, 2 * (1 << 20) + 65536, dtype=np.uint8).tobytes()]


def test_single_object_parallel_stage_matches_oracle(ca):
    """encode()'s single-object Ecies|Snappy stage from 256 KiB up runs its
    snappy blocks on a few threads and AES-GCM on the caller in block order
    (host_stages.cpp ecies_encrypt_par): byte-identical to the C oracle's
    snap + ecies with the injected ephemeral key and nonce, at and around the
    threshold, compressible and not, and it round-trips with fresh
    randomness."""
    sk = H.sha256(b"par receiver")
    pub = H.public_key(sk)
    eph, nonce = H.sha256(b"par eph"), H.sha256(b"par nonce")[:16]
    for d in _par_inputs():
        enc, h, info = ca.encode(pub, d, 3, ephemeral_sk=eph, nonce=nonce)
        oenc, oh, oinfo = O.c_encode_full(d, 3, pub, eph, nonce)
        assert enc == oenc, len(d)
        assert info.bytes_compressed == oinfo["bytes_compressed"]
        assert ca.decode(sk, h, enc, info.padding_len, 3) == d
        fresh, h2, info2 = ca.encode(pub, d, 3)
        assert fresh[:97] != enc[:97] and ca.decode(sk, h2, fresh, info2.padding_len, 3) == d


def test_single_object_parallel_gcm_without_snappy(ca):
    """Ecies alone (level 1) from 256 KiB: AES-GCM split over the stage pool
    (ecies_encrypt_par_plain / ecies_decrypt_par): the C oracle's envelope,
    a flipped tag or ciphertext byte refused, fresh randomness round-trips."""
    from carbonado_amd.error import EciesError
    sk = H.sha256(b"par receiver")
    pub = H.public_key(sk)
    eph, nonce = H.sha256(b"plain eph"), H.sha256(b"plain nonce")[:16]
    for d in _par_inputs():
        enc, h, info = ca.encode(pub, d, 1, ephemeral_sk=eph, nonce=nonce)
        assert enc == O.c_encode_full(d, 1, pub, eph, nonce)[0], len(d)
        assert ca.decode(sk, h, enc, info.padding_len, 1) == d
        for pos in (81, 96, 97, len(enc) // 2, len(enc) - 1):
            bad = bytearray(enc)
            bad[pos] ^= 4
            with pytest.raises(EciesError):
                ca.decode(sk, h, bytes(bad), info.padding_len, 1)
        fresh, h2, info2 = ca.encode(pub, d, 1)
        assert ca.decode(sk, h2, fresh, info2.padding_len, 1) == d


def test_single_object_stage_concurrent_callers(ca):
    """Several threads calling encode() at once: one gets the stage's worker
    pool, the others take the one-thread path; every output is the oracle's."""
    from concurrent.futures import ThreadPoolExecutor
    sk = H.sha256(b"par receiver")
    pub = H.public_key(sk)
    ins = _par_inputs()[1:]
    jobs = [(d, H.sha256(b"eph %d" % i), H.sha256(b"nonce %d" % i)[:16]) for i, d in enumerate(ins * 3)]

    def run(job):
        d, e, nn = job
        return ca.encode(pub, d, 3, ephemeral_sk=e, nonce=nn)[0]

    with ThreadPoolExecutor(6) as ex:
        outs = list(ex.map(run, jobs))
    for (d, e, nn), got in zip(jobs, outs):
        assert got == O.c_encode_full(d, 3, pub, e, nn)[0]


@pytest.mark.parametrize("level", [1, 3])
def test_decode_host_batch_host_only_levels(ca, level):
    """chip_decode_host_batch at host-only levels (no device part) decodes
    object by object, each large one on the stage pool: every object back,
    a tampered envelope fails alone with EciesError's status."""
    import torch
    from carbonado_amd import device
    sk = H.sha256(b"par receiver")
    pub = H.public_key(sk)
    ins = _par_inputs()[:4]
    encs = [ca.encode(pub, d, level)[0] for d in ins]
    width = max(len(e) for e in encs)
    enc = torch.zeros((len(encs), width), dtype=torch.uint8)
    for i, e in enumerate(encs):
        enc[i, :len(e)] = torch.frombuffer(bytearray(e), dtype=torch.uint8)
    out = torch.zeros((len(encs), max(len(d) for d in ins) + 64), dtype=torch.uint8)
    hashes = torch.zeros((len(encs), 32), dtype=torch.uint8)
    lens, pads = [len(e) for e in encs], [0] * len(encs)
    dlen, st = device.decode_host_batch(level, enc, lens, hashes, pads, out, secret_key=sk)
    assert st == [0] * len(encs)
    for i, d in enumerate(ins):
        assert dlen[i] == len(d) and out[i, :len(d)].numpy().tobytes() == d
    enc[1, lens[1] - 1] ^= 1
    out.zero_()
    dlen, st = device.decode_host_batch(level, enc, lens, hashes, pads, out, secret_key=sk, raise_first=False)
    assert st[1] != 0 and st[0] == st[2] == st[3] == 0
    assert not out[1].any()  # the failed object's plaintext was wiped
    for i in (0, 2, 3):
        assert out[i, :len(ins[i])].numpy().tobytes() == ins[i]


def test_compressed_receiver_keys(ca):
    """33-byte receiver keys are decompressed by the native field code
    (secp256k1_host.hpp decompress: x < p, y = (x^3 + 7)^((p+1)/4) checked,
    the tag's parity): the same envelope as with the 65-byte key for 64
    random receivers, and EciesError for x >= p, an x off the curve and
    other tags."""
    from carbonado_amd.error import EciesError
    P = 2**256 - 2**32 - 977
    eph, nonce = H.sha256(b"cmp eph"), H.sha256(b"cmp nonce")[:16]
    msg = b"compressed receiver " * 50
    for i in range(64):
        pub = H.public_key(H.sha256(b"cmp %d" % i))
        x, y = int.from_bytes(pub[1:33], "big"), int.from_bytes(pub[33:], "big")
        pk33 = bytes([2 + (y & 1)]) + pub[1:33]
        assert ca.encoding.ecies(pk33, msg, ephemeral_sk=eph, nonce=nonce) == H.ecies_encrypt(pub, msg, eph, nonce)
    off = next(x for x in range(1, 100) if pow((x**3 + 7) % P, (P - 1) // 2, P) != 1)
    bad = [b"\x02" + P.to_bytes(32, "big"), b"\x03" + (P + 5).to_bytes(32, "big"),
           b"\x02" + off.to_bytes(32, "big"), b"\x04" + pub[1:33], b"\x05" + pub[1:33], b"\x00" * 33]
    for pk in bad:
        with pytest.raises(EciesError):
            ca.encoding.ecies(pk, msg, ephemeral_sk=eph, nonce=nonce)


def test_uncompressed_keys_checked_natively(ca):
    """65- and 64-byte keys (the receiver's on encrypt, the envelope's
    ephemeral one on decrypt) are parsed by the native field code
    (secp256k1_host.hpp parse_full: x, y < p and y^2 = x^3 + 7), as
    PublicKey::parse_slice accepts them: the C oracle's envelope for valid
    keys, EciesError for a point off the curve or a coordinate >= p; the
    hybrid 0x06 / 0x07 forms (OpenSSL's route) give the 0x04 form's envelope
    with the right parity tag and EciesError with the wrong one."""
    from carbonado_amd.error import EciesError
    P = 2**256 - 2**32 - 977
    sk = H.sha256(b"full receiver")
    pub = H.public_key(sk)
    x, y = int.from_bytes(pub[1:33], "big"), int.from_bytes(pub[33:], "big")
    eph, nonce = H.sha256(b"full eph"), H.sha256(b"full nonce")[:16]
    msg = b"uncompressed receiver " * 40
    good = H.ecies_encrypt(pub, msg, eph, nonce)
    assert ca.encoding.ecies(pub, msg, ephemeral_sk=eph, nonce=nonce) == good
    assert ca.encoding.ecies(pub[1:], msg, ephemeral_sk=eph, nonce=nonce) == good
    hyb = bytes([6 + (y & 1)]) + pub[1:]
    assert ca.encoding.ecies(hyb, msg, ephemeral_sk=eph, nonce=nonce) == good
    pt = lambda a, b: b"\x04" + a.to_bytes(32, "big") + b.to_bytes(32, "big")
    bad = [pt(x, (y + 1) % P), pt(x, P - y + 1), bytes([7 - (y & 1)]) + pub[1:], b"\x05" + pub[1:],
           b"\x04" + bytes(64), pt((x + 1) % P, y)]
    if y + P < 2**256:
        bad.append(pt(x, y + P))
    if x + P < 2**256:
        bad.append(pt(x + P, y))
    for pk in bad + [b[1:] for b in bad if b[0] == 4]:
        with pytest.raises(EciesError):
            ca.encoding.ecies(pk, msg, ephemeral_sk=eph, nonce=nonce)
    assert ca.decoding.ecies(good, sk) == msg
    ex, ey = int.from_bytes(good[1:33], "big"), int.from_bytes(good[33:65], "big")
    for e65 in [pt(ex, (ey + 1) % P), pt(ex, P), b"\x04" + bytes(64)] + ([pt(ex, ey + P)] if ey + P < 2**256 else []):
        with pytest.raises(EciesError):
            ca.decoding.ecies(e65 + good[65:], sk)


@pytest.mark.parametrize("n", [256 * 1024 - 97, 256 * 1024, 300_001, 5 << 20])
def test_ecies_stage_functions_on_the_pool_match_oracle(ca, n):
    """chip_ecies_encrypt / chip_ecies_decrypt (the stage functions) split a
    large message's AES-GCM over the stage pool (host_stages_par.cpp,
    ecies_encrypt_par_plain / ecies_decrypt_par, from STAGE_PAR_MIN = 256 KiB):
    the envelope is byte-identical to the C oracle's with the same injected
    key and nonce, it decrypts back, and a flipped ciphertext byte is refused
    with the written plaintext wiped."""
    from carbonado_amd.error import EciesError
    sk = H.sha256(b"pool receiver")
    pub = ca.encoding.public_key(sk)
    eph, nonce = H.sha256(b"pool eph"), H.sha256(b"pool nonce")[:16]
    d = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    e = ca.encoding.ecies(pub, d, ephemeral_sk=eph, nonce=nonce)
    assert e == O.c_ecies_encrypt(pub, d, eph, nonce)
    assert ca.decoding.ecies(e, sk) == d == O.c_ecies_decrypt(sk, e)
    bad = bytearray(e)
    bad[len(bad) // 2] ^= 1
    with pytest.raises(EciesError):
        ca.decoding.ecies(bytes(bad), sk)


def test_ecies_receiver_comb_tables_match_oracle(ca):
    """ecies_prepare's ECDH for a receiver key seen before runs on a comb table
    built for that key (host_stages.cpp peer_mul, from its second use; at most
    8 receivers kept, least recently used replaced): the envelopes stay
    byte-identical to the C oracle's for 11 receivers interleaved over many
    rounds (first uses, table hits, evictions and rebuilds), both key forms."""
    rng = np.random.default_rng(77)
    receivers = []
    for i in range(11):
        sk = H.sha256(b"comb receiver %d" % i)
        receivers.append((sk, ca.encoding.public_key(sk)))
    order = [i % 11 for i in range(60)] + list(rng.integers(0, 11, 60))
    for r, i in enumerate(order):
        sk, pub = receivers[int(i)]
        eph = H.sha256(b"comb eph %d" % r)
        nonce = H.sha256(b"comb nonce %d" % r)[:16]
        d = rng.integers(0, 256, 100 + r, dtype=np.uint8).tobytes()
        pk = pub if r % 3 else (b"\x02" if H.parse_pubkey(pub)[1] % 2 == 0 else b"\x03") + pub[1:33]
        e = ca.encoding.ecies(pk, d, ephemeral_sk=eph, nonce=nonce)
        assert e == O.c_ecies_encrypt(pub, d, eph, nonce), (r, int(i))
        assert ca.decoding.ecies(e, sk) == d


@pytest.mark.parametrize("kind", ["random", "text", "mixed"])
def test_snap_stage_functions_on_the_pool_match_oracle(ca, kind):
    """chip_snap_compress / chip_snap_decompress (and the Snappy stage of a
    single encode()/decode()) split an input of 256 KiB or more into its
    64 KiB blocks on the stage pool (host_stages_par.cpp snap_compress_par /
    snap_decompress_par): the frame is byte-identical to the C oracle's, it
    decodes back, a flipped byte is refused."""
    rng = np.random.default_rng({"random": 1, "text": 2, "mixed": 3}[kind])
    n = (1 << 20) + 12345
    if kind == "random":
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    else:
        words = [b"carbonado ", b"segment ", b"zfec ", b"bao ", b"{\"id\": ", b"\n"]
        d = b"".join(rng.choice(words, n // 4).tolist())[:n]
        if kind == "mixed":  # incompressible stretches between the text
            a = bytearray(d)
            for o in range(0, n - 70_000, 200_000):
                a[o:o + 70_000] = rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes()
            d = bytes(a)
    f = ca.encoding.snap(d)
    assert f == O.c_snap_compress(d)
    assert ca.decoding.snap(f) == d
    bad = bytearray(f)
    bad[len(bad) // 2] ^= 0x10
    with pytest.raises(Exception):
        ca.decoding.snap(bytes(bad))
