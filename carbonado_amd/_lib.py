"""ctypes binding of libcarbonado_hip.so (include/carbonado_hip.h).

The shared library is the product: HIP kernels for gfx950 behind a C-ABI.
This module only loads it and declares signatures.  There is no fallback:
if the library is missing, or no gfx950 device is visible, compute calls
raise instead of silently running elsewhere.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

# CARBONADO_HIP_LIB: another build of the same library (A/B calibration tools only)
LIB_PATH = Path(os.environ.get("CARBONADO_HIP_LIB") or Path(__file__).resolve().parent / "lib" / "libcarbonado_hip.so")

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


class EncodeInfoC(ctypes.Structure):
    """chip_encode_info == structs.rs:12-44 EncodeInfo, field for field."""

    _fields_ = [
        ("input_len", ctypes.c_uint32),
        ("output_len", ctypes.c_uint32),
        ("bytes_compressed", ctypes.c_uint32),
        ("compression_factor", ctypes.c_float),
        ("bytes_encrypted", ctypes.c_uint32),
        ("bytes_ecc", ctypes.c_uint32),
        ("bytes_verifiable", ctypes.c_uint32),
        ("amplification_factor", ctypes.c_float),
        ("padding_len", ctypes.c_uint32),
        ("chunk_len", ctypes.c_uint32),
        ("verifiable_slice_count", ctypes.c_uint16),
        ("chunk_slice_count", ctypes.c_uint16),
    ]


class EciesInjectC(ctypes.Structure):
    """chip_ecies_inject: the values ecies::encrypt draws from thread_rng."""

    _fields_ = [("ephemeral_sk", ctypes.c_void_p), ("nonce", ctypes.c_void_p)]


class HeaderC(ctypes.Structure):
    """chip_header == file.rs:24-43 Header, deserialized."""

    _fields_ = [
        ("pubkey", ctypes.c_uint8 * 33),
        ("hash", ctypes.c_uint8 * 32),
        ("signature", ctypes.c_uint8 * 64),
        ("format", ctypes.c_uint8),
        ("chunk_index", ctypes.c_uint8),
        ("encoded_len", ctypes.c_uint32),
        ("padding_len", ctypes.c_uint32),
        ("metadata", ctypes.c_uint8 * 8),
        ("has_metadata", ctypes.c_uint8),
    ]


# name -> (restype, argtypes); mirrors include/carbonado_hip.h exactly
SIGNATURES = {
    "chip_abi_version": (ctypes.c_int, []),
    "chip_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "chip_init": (ctypes.c_int, [ctypes.c_int]),
    "chip_last_device_error": (ctypes.c_char_p, []),
    "chip_device_alloc": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "chip_device_free": (ctypes.c_int, [ctypes.c_void_p]),
    "chip_schnorr_sign": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "chip_schnorr_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "chip_header_new": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint8, ctypes.c_uint8,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.POINTER(HeaderC)]),
    "chip_header_to_bytes": (ctypes.c_int, [ctypes.POINTER(HeaderC), ctypes.c_void_p]),
    "chip_header_parse": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(HeaderC)]),
    "chip_file_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint8, ctypes.c_void_p,
                                        ctypes.POINTER(EciesInjectC), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint64, c_u64p, ctypes.POINTER(EncodeInfoC)]),
    "chip_file_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.POINTER(HeaderC), ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_device_alloc_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_double)]),
    "chip_stream_queue_block": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "chip_host_topology": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "chip_torch_alloc": (ctypes.c_void_p, [ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]),
    "chip_torch_free": (None, [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]),
    "chip_calc_padding_len": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, c_u32p, c_u32p]),
    "chip_zfec_encoded_len": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]),
    "chip_bao_encoded_len": (ctypes.c_uint64, [ctypes.c_uint64]),
    "chip_encode_max_len": (ctypes.c_uint64, [ctypes.c_uint64]),
    "chip_zfec_encode": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_uint64, c_u32p, c_u32p]),
    "chip_zfec_decode": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_zfec_decode_shares": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_void_p), c_u32p, ctypes.c_uint32,
                                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                               ctypes.c_uint64, c_u64p]),
    "chip_bao_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                       c_u64p, ctypes.c_void_p]),
    "chip_bao_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_blake3": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "chip_snap_max_len": (ctypes.c_uint64, [ctypes.c_uint64]),
    "chip_snap_compress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                          c_u64p]),
    "chip_snap_decompress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                            c_u64p]),
    "chip_ecies_encrypt": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(EciesInjectC),
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                          c_u64p]),
    "chip_ecies_decrypt": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_ecies_public_key": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "chip_encode": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(EciesInjectC),
                                   ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, c_u64p,
                                   ctypes.c_void_p, ctypes.POINTER(EncodeInfoC)]),
    "chip_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint8,
                                   ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_zfec_encode_batch_dev": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "chip_hbm_pattern_batch_dev": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "chip_zfec_decode_batch_dev": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                  ctypes.c_uint64, ctypes.c_uint64, c_u32p, ctypes.c_uint32,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                  ctypes.c_void_p]),
    "chip_bao_scratch_len": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    "chip_bao_encode_batch_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "chip_bao_decode_batch_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "chip_encode_scratch_len": (ctypes.c_uint64, [ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint64]),
    "chip_encode_batch_dev": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, c_u64p,
                                             ctypes.c_void_p, ctypes.POINTER(EncodeInfoC), ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "chip_decode_scratch_len": (ctypes.c_uint64, [ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint64]),
    "chip_decode_batch_dev": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                             ctypes.c_uint64, c_u64p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    "chip_bao_slice_len": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "chip_bao_extract_slice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_bao_verify_slice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                             c_u64p]),
    "chip_scrub": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_scrub_scratch_len": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
    "chip_scrub_batch_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "chip_bao_hasher_new": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "chip_bao_hasher_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "chip_bao_hasher_finalize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "chip_bao_hasher_len": (ctypes.c_uint64, [ctypes.c_void_p]),
    "chip_bao_hasher_read_all": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, c_u64p]),
    "chip_bao_hasher_free": (None, [ctypes.c_void_p]),
    "chip_bao_hasher_drop_cache": (ctypes.c_uint64, []),
    "chip_bao_hasher_cached_bytes": (ctypes.c_uint64, []),
    "chip_decode_host_batch": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_void_p, c_u64p, ctypes.c_uint64, ctypes.c_uint64, c_u32p,
                                              ctypes.c_void_p, ctypes.c_uint64, c_u64p,
                                              ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, ctypes.c_uint64,
                                              ctypes.c_uint32]),
    "chip_encode_host_batch": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.POINTER(EciesInjectC), ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                              c_u64p, ctypes.c_void_p, ctypes.POINTER(EncodeInfoC),
                                              ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]),
}

_LIB = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is not built."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the carbonado hot path)")
        # One HIP runtime per process.  torch's HIP libs NEED "libamdhip64.so"
        # (unversioned, RPATH $ORIGIN) while this library NEEDs the soname
        # "libamdhip64.so.7": loading torch first makes both bind to torch's
        # copy; the reverse order would map two runtimes.
        try:
            import torch  # noqa: F401
        except ImportError:  # torch is plumbing only; the library does not need it
            pass
        l = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = l
    return _LIB
