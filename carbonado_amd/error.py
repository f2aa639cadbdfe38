"""CarbonadoError (mirror of /root/reference/src/error.rs, hot-path variants).

Each C-ABI status code maps to the variant the reference would return for
the same condition; `status_to_error` is the single place that mapping lives.
"""
from __future__ import annotations


class CarbonadoError(Exception):
    """error.rs:4 `pub enum CarbonadoError`."""

    status: int = -1


class UnevenZfecChunks(CarbonadoError):
    """error.rs:61-63"""
    status = 3

    def __init__(self, msg="Input bytes must divide evenly over number of zfec chunks."):
        super().__init__(msg)


class HashDecodeError(CarbonadoError):
    """error.rs:77-79 HashDecodeError(expected, got)"""
    status = 4

    def __init__(self, expected: int = 32, got: int = -1):
        super().__init__(f"Hash must be {expected} bytes long, an input of {got} bytes was provided.")
        self.expected, self.got = expected, got


class BaoDecodeError(CarbonadoError):
    """error.rs:45-47 BaoDecodeError(bao::decode::Error) — HashMismatch or Truncated."""
    status = 5

    def __init__(self, kind: str = "HashMismatch"):
        super().__init__(f"bao decode error: {kind}")
        self.kind = kind


class ZfecError(CarbonadoError):
    """error.rs:49-51 ZfecError(zfec_rs::Error)"""
    status = 7


class EncodeZfecPaddingError(CarbonadoError):
    """error.rs:85-87"""
    status = 8


class EncodeInvalidChunkLength(CarbonadoError):
    """error.rs:89-91"""
    status = 9


class InvalidVerifiableSliceCount(CarbonadoError):
    """error.rs:93-95"""
    status = 10


class UnsupportedFormat(CarbonadoError):
    """Reserved status (ABI 1 rejected the Ecies/Snappy bits with it)."""
    status = 11


class SnapError(CarbonadoError):
    """error.rs:7,35 StdIoError / SnapError: FrameDecoder rejected the stream."""
    status = 16


class EciesError(CarbonadoError):
    """error.rs:43 EciesError: bad key, short input or AES-GCM tag mismatch."""
    status = 17


class Secp256k1Error(CarbonadoError):
    """error.rs:55 NostrSecp256k1Error(secp256k1::Error): bad key, message or
    Schnorr signature (Header::new / Header::try_from, file.rs:263-289, :116-154)."""
    status = 18


class InvalidHeaderLength(CarbonadoError):
    """error.rs:113-115 (also a header slice too short to parse, where the
    reference panics, file.rs:126)"""
    status = 19


class InvalidMagicNumber(CarbonadoError):
    """error.rs:97-99"""
    status = 20


class UnnecessaryScrub(CarbonadoError):
    """error.rs:65-67"""
    status = 12

    def __init__(self, msg="Data does not need to be scrubbed."):
        super().__init__(msg)


class ScrubbedPaddingMismatch(CarbonadoError):
    """error.rs:69-71"""
    status = 13


class ScrubbedLengthMismatch(CarbonadoError):
    """error.rs:73-75"""
    status = 14


class InvalidScrubbedHash(CarbonadoError):
    """error.rs:81-83"""
    status = 15


class BufferTooSmall(CarbonadoError):
    status = 2


class InvalidArgument(CarbonadoError):
    status = 1


class DeviceError(CarbonadoError):
    """New variant: HIP runtime failure or no gfx950 device (no CPU fallback)."""
    status = 101


def status_to_error(status: int, detail: str = "") -> CarbonadoError:
    if status == 3:
        return UnevenZfecChunks()
    if status == 4:
        return HashDecodeError(32, -1)
    if status == 5:
        return BaoDecodeError("HashMismatch")
    if status == 6:
        return BaoDecodeError("Truncated")
    if status == 7:
        return ZfecError("zfec error" + (f": {detail}" if detail else ""))
    if status == 8:
        return EncodeZfecPaddingError("zfec padding should always be zero")
    if status == 9:
        return EncodeInvalidChunkLength("chunk length should be as calculated")
    if status == 10:
        return InvalidVerifiableSliceCount("Verifiable slice count should be evenly divisible by 8.")
    if status == 11:
        return UnsupportedFormat("unsupported format")
    if status == 16:
        return SnapError("snappy framing error")
    if status == 17:
        return EciesError("ecies error")
    if status == 18:
        return Secp256k1Error("secp256k1 error (key, message or signature)")
    if status == 19:
        return InvalidHeaderLength("Invalid header length calculation")
    if status == 20:
        return InvalidMagicNumber("File header lacks Carbonado magic number and may not be a proper Carbonado file.")
    if status == 12:
        return UnnecessaryScrub()
    if status == 13:
        return ScrubbedPaddingMismatch("Scrubbed padding should remain the same.")
    if status == 14:
        return ScrubbedLengthMismatch("Mismatch between scrubbed data length and input length")
    if status == 15:
        return InvalidScrubbedHash("Scrubbed hash is not equal to original hash.")
    if status == 2:
        return BufferTooSmall("output buffer too small")
    if status == 1:
        return InvalidArgument("invalid argument")
    if status in (100, 101):
        e = DeviceError(("no usable gfx950 device" if status == 100 else "HIP runtime error")
                        + (f": {detail}" if detail else ""))
        e.status = status
        return e
    return CarbonadoError(f"status {status}")
