"""GPU: the flat-file container at the device levels (zfec + bao on the
MI355X): tests/format.rs restated (a level-15 file written to disk, its header
parsed from the file, the body decoded), file::encode bytes against the oracle
on the reference's samples, and tampering caught by the header signature or
by bao."""
import pytest

from oracle import host_oracle as H
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SAMPLES = ["contract.rgbc", "content.png", "code.tar"]


def test_format_rs_restated(gpu, tmp_path):
    """tests/format.rs:16-95: encode "Hello world!" at level 15, header with
    encoded_len = bytes_verifiable, write header + body to <hash>.c15, parse
    the header back from the file, check its fields, decode the body."""
    import carbonado_amd as ca
    from carbonado_amd.file import Header
    file_sk, node_sk = H.sha256(b"format file sk"), H.sha256(b"format node sk")
    # the test's key: an ECDH shared secret of two keypairs (format.rs:24-39)
    shared = H.point_mul(int.from_bytes(node_sk, "big"), H.parse_pubkey(H.public_key(file_sk)))
    sk = H.sha256(H.ser_compressed(shared))
    pk = H.ser_compressed(H.parse_pubkey(H.public_key(sk)))
    data = b"Hello world!"
    enc, h, info = ca.encode(pk, data, 15)
    header = Header.new(sk, pk, h, 15, 0, info.bytes_verifiable, info.padding_len, None)
    path = tmp_path / header.file_name()
    path.write_bytes(header.try_to_vec() + enc)
    back = Header.from_file(path)
    assert back.pubkey == pk and back.hash == h and back.format == 15 and back.chunk_index == 0
    assert back.padding_len == info.padding_len and back.encoded_len == info.bytes_verifiable
    assert ca.decode(sk, h, path.read_bytes()[160:], info.padding_len, 15) == data


@pytest.mark.parametrize("name", SAMPLES)
@pytest.mark.parametrize("level", [4, 8, 12, 14, 15])
def test_file_encode_samples_bit_exact(gpu, golden_dir, name, level):
    from carbonado_amd import file
    sk = H.sha256(b"file sample sk")
    eph, nonce, aux = H.sha256(b"fs eph"), H.sha256(b"fs nonce")[:16], H.sha256(b"fs aux")
    data = (golden_dir / "samples" / name).read_bytes()
    out, info = file.encode(sk, None, data, level, b"\x00\x00\x00\x00\x00\x00\x00\x07", ephemeral_sk=eph,
                            nonce=nonce, aux_rand=aux)
    pub33 = H.ser_compressed(H.parse_pubkey(H.public_key(sk)))
    body, h, oinfo = O.c_encode_full(data, level, pub33, eph, nonce)
    want = H.header_bytes(sk, pub33, h, level, 0, oinfo["output_len"], oinfo["padding_len"],
                          b"\x00\x00\x00\x00\x00\x00\x00\x07", aux) + body
    assert out == want
    hdr, back = file.decode(sk, out)
    assert back == data and hdr.metadata == b"\x00\x00\x00\x00\x00\x00\x00\x07"
    assert hdr.encoded_len == info.output_len == len(body)


def test_file_tampering(gpu, golden_dir):
    from carbonado_amd import file
    from carbonado_amd.error import BaoDecodeError, InvalidHeaderLength, Secp256k1Error
    sk = H.sha256(b"tamper sk")
    data = (golden_dir / "samples" / "code.tar").read_bytes()
    out, _ = file.encode(sk, None, data, 12)
    bad = bytearray(out)
    bad[60] ^= 1  # the hash in the header: the signature no longer verifies
    with pytest.raises(Secp256k1Error):
        file.decode(sk, bytes(bad))
    bad = bytearray(out)
    bad[160 + 5000] ^= 1  # the body: bao catches it
    with pytest.raises(BaoDecodeError):
        file.decode(sk, bytes(bad))
    with pytest.raises(InvalidHeaderLength):
        file.decode(sk, out[:100])
