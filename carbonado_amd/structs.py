"""EncodeInfo / Encoded (mirror of /root/reference/src/structs.rs:11-48)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import NamedTuple


@dataclass
class EncodeInfo:
    """structs.rs:12-44, same fields and integer widths (u32 / f32 / u16)."""

    input_len: int
    output_len: int
    bytes_compressed: int
    compression_factor: float
    bytes_encrypted: int
    bytes_ecc: int
    bytes_verifiable: int
    amplification_factor: float
    padding_len: int
    chunk_len: int
    verifiable_slice_count: int
    chunk_slice_count: int

    @classmethod
    def from_c(cls, c) -> "EncodeInfo":
        return cls(**{name: getattr(c, name) for name, _ in c._fields_})


class Encoded(NamedTuple):
    """structs.rs:46-48 `Encoded(Vec<u8>, bao::Hash, EncodeInfo)`."""

    data: bytes
    hash: bytes
    info: EncodeInfo
