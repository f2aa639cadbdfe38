"""Constants of the hot path (mirror of /root/reference/src/constants.rs)."""
from enum import IntFlag

#: constants.rs:5 — file-format magic number (the container itself is out of scope)
MAGICNO = b"CARBONADO01\n"
#: constants.rs:9 — bao slice length
SLICE_LEN = 1024
#: constants.rs:11 — zfec chunks needed (k)
FEC_K = 4
#: constants.rs:13 — zfec chunks encoded (m)
FEC_M = 8
#: bao::HASH_SIZE
HASH_SIZE = 32


class Format(IntFlag):
    """constants.rs:49-56 — `#[bitmask(u8)]` in declaration order."""

    Ecies = 1
    Snappy = 2
    Bao = 4
    Zfec = 8

    def contains(self, other: "Format") -> bool:
        return (self & other) == other
