"""carbonado_amd — MI355X-native (gfx950) hot path of carbonado's
encode()/decode(): zfec erasure coding and bao/BLAKE3 verifiable streams.

Mirrors the reference crate's public surface for this path
(/root/reference/src/lib.rs:21-29): `encode`, `decode`, plus the stage
functions in `encoding` / `decoding`.  Compute happens only in
`lib/libcarbonado_hip.so` (HIP kernels); see DESIGN.md.
"""
from . import constants, decoding, encoding, error, file, structs, utils
from .constants import FEC_K, FEC_M, HASH_SIZE, SLICE_LEN, Format
from .decoding import decode, extract_slice, scrub, verify_slice
from .encoding import encode
from .error import CarbonadoError
from .structs import EncodeInfo, Encoded

__all__ = [
    "encode", "decode", "extract_slice", "verify_slice", "scrub", "Encoded", "EncodeInfo", "Format", "CarbonadoError",
    "FEC_K", "FEC_M", "SLICE_LEN", "HASH_SIZE",
    "constants", "decoding", "encoding", "error", "file", "structs", "utils",
]
