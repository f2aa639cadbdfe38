//! Raw bindings of `include/carbonado_hip.h` (ABI 5), one declaration per
//! `CHIP_API` prototype, in the header's order.  Kept in lock-step with the
//! header by `tests/test_rust_shim.py` (name, arity, C <-> Rust type of every
//! parameter and return value, struct layouts, constants).
//!
//! The C `in` parameter is spelled `input` here (`in` is a Rust keyword);
//! array parameters (`uint8_t hash[32]`) decay to pointers, as in C.
#![allow(non_camel_case_types)]
#![allow(dead_code)]

use std::os::raw::{c_char, c_int, c_void};

pub const CHIP_ABI_VERSION: c_int = 5;
pub const CHIP_HASH_LEN: usize = 32; // bao::HASH_SIZE
pub const CHIP_SLICE_LEN: usize = 1024; // constants.rs:9 SLICE_LEN
pub const CHIP_FEC_K: u32 = 4; // constants.rs:11 FEC_K
pub const CHIP_FEC_M: u32 = 8; // constants.rs:13 FEC_M
pub const CHIP_HEADER_LEN: usize = 160; // file.rs:257-259 Header::len()

pub const CHIP_FORMAT_ECIES: u8 = 1;
pub const CHIP_FORMAT_SNAPPY: u8 = 2;
pub const CHIP_FORMAT_BAO: u8 = 4;
pub const CHIP_FORMAT_ZFEC: u8 = 8;

// enum chip_status (the values returned by every entry point)
pub const CHIP_OK: c_int = 0;
pub const CHIP_ERR_INVALID_ARG: c_int = 1;
pub const CHIP_ERR_BUFFER_TOO_SMALL: c_int = 2;
pub const CHIP_ERR_UNEVEN_ZFEC_CHUNKS: c_int = 3;
pub const CHIP_ERR_HASH_DECODE: c_int = 4;
pub const CHIP_ERR_BAO_HASH_MISMATCH: c_int = 5;
pub const CHIP_ERR_BAO_TRUNCATED: c_int = 6;
pub const CHIP_ERR_ZFEC: c_int = 7;
pub const CHIP_ERR_ENCODE_ZFEC_PADDING: c_int = 8;
pub const CHIP_ERR_ENCODE_INVALID_CHUNK_LENGTH: c_int = 9;
pub const CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT: c_int = 10;
pub const CHIP_ERR_UNSUPPORTED_FORMAT: c_int = 11;
pub const CHIP_ERR_UNNECESSARY_SCRUB: c_int = 12;
pub const CHIP_ERR_SCRUBBED_PADDING_MISMATCH: c_int = 13;
pub const CHIP_ERR_SCRUBBED_LENGTH_MISMATCH: c_int = 14;
pub const CHIP_ERR_INVALID_SCRUBBED_HASH: c_int = 15;
pub const CHIP_ERR_SNAP: c_int = 16;
pub const CHIP_ERR_ECIES: c_int = 17;
pub const CHIP_ERR_SECP256K1: c_int = 18;
pub const CHIP_ERR_INVALID_HEADER_LENGTH: c_int = 19;
pub const CHIP_ERR_INVALID_MAGIC: c_int = 20;
pub const CHIP_ERR_NO_DEVICE: c_int = 100;
pub const CHIP_ERR_DEVICE: c_int = 101;

/// structs.rs:12-44 EncodeInfo, field for field.
#[repr(C)]
#[derive(Default, Clone, Copy, Debug, PartialEq)]
pub struct chip_encode_info {
    pub input_len: u32,
    pub output_len: u32,
    pub bytes_compressed: u32,
    pub compression_factor: f32,
    pub bytes_encrypted: u32,
    pub bytes_ecc: u32,
    pub bytes_verifiable: u32,
    pub amplification_factor: f32,
    pub padding_len: u32,
    pub chunk_len: u32,
    pub verifiable_slice_count: u16,
    pub chunk_slice_count: u16,
}

/// The two values ecies::encrypt draws from thread_rng; null = random.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct chip_ecies_inject {
    pub ephemeral_sk: *const u8,
    pub nonce: *const u8,
}

/// file.rs:24-43 Header, deserialized.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct chip_header {
    pub pubkey: [u8; 33],
    pub hash: [u8; 32],
    pub signature: [u8; 64],
    pub format: u8,
    pub chunk_index: u8,
    pub encoded_len: u32,
    pub padding_len: u32,
    pub metadata: [u8; 8],
    pub has_metadata: u8,
}

impl Default for chip_header {
    fn default() -> Self {
        chip_header {
            pubkey: [0; 33],
            hash: [0; 32],
            signature: [0; 64],
            format: 0,
            chunk_index: 0,
            encoded_len: 0,
            padding_len: 0,
            metadata: [0; 8],
            has_metadata: 0,
        }
    }
}

/// Opaque streaming hasher (utils.rs:104-137 BaoHasher).
#[repr(C)]
pub struct chip_bao_hasher {
    _private: [u8; 0],
}

extern "C" {
    // ---- library
    pub fn chip_abi_version() -> c_int;
    pub fn chip_strerror(status: c_int) -> *const c_char;
    pub fn chip_init(device: c_int) -> c_int;
    pub fn chip_last_device_error() -> *const c_char;

    // ---- flat-file container (file.rs)
    pub fn chip_schnorr_sign(sk: *const u8, sk_len: u64, msg32: *const u8, aux32: *const u8, sig64: *mut u8)
        -> c_int;
    pub fn chip_schnorr_verify(pubkey: *const u8, pubkey_len: u64, msg32: *const u8, sig64: *const u8) -> c_int;
    pub fn chip_header_new(sk: *const u8, sk_len: u64, pk: *const u8, pk_len: u64, hash: *const u8,
                           hash_len: u64, format: u8, chunk_index: u8, encoded_len: u32, padding_len: u32,
                           metadata8: *const u8, aux32: *const u8, out: *mut chip_header) -> c_int;
    pub fn chip_header_to_bytes(h: *const chip_header, out160: *mut u8) -> c_int;
    pub fn chip_header_parse(bytes: *const u8, len: u64, out: *mut chip_header) -> c_int;
    pub fn chip_file_encode(sk: *const u8, sk_len: u64, pk: *const u8, pk_len: u64, input: *const u8, n: u64,
                            level: u8, metadata8: *const u8, inject: *const chip_ecies_inject, aux32: *const u8,
                            out: *mut u8, out_cap: u64, out_len: *mut u64, info: *mut chip_encode_info) -> c_int;
    pub fn chip_file_decode(sk: *const u8, sk_len: u64, input: *const u8, n: u64, hdr: *mut chip_header,
                            out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;

    // ---- batch buffers
    pub fn chip_device_alloc(bytes: u64, ptr: *mut *mut c_void) -> c_int;
    pub fn chip_device_free(ptr: *mut c_void) -> c_int;
    pub fn chip_device_alloc_info(ptr: *const c_void, classes_found: *mut u32, classes_used: *mut u32,
                                  seconds: *mut f64) -> c_int;
    pub fn chip_torch_alloc(size: isize, device: c_int, stream: *mut c_void) -> *mut c_void;
    pub fn chip_torch_free(ptr: *mut c_void, size: isize, device: c_int, stream: *mut c_void);
    pub fn chip_stream_queue_block(stream: *mut c_void, addr: *mut u64) -> c_int;
    pub fn chip_host_topology(json: *mut c_char, cap: u64, len: *mut u64) -> c_int;

    // ---- size helpers (host only)
    pub fn chip_calc_padding_len(input_len: u64, k: u32, padding: *mut u32, chunk_len: *mut u32) -> c_int;
    pub fn chip_zfec_encoded_len(input_len: u64, k: u32, m: u32) -> u64;
    pub fn chip_bao_encoded_len(content_len: u64) -> u64;
    pub fn chip_encode_max_len(input_len: u64) -> u64;
    pub fn chip_snap_max_len(input_len: u64) -> u64;

    // ---- stage functions (host buffers)
    pub fn chip_zfec_encode(k: u32, m: u32, input: *const u8, n: u64, out: *mut u8, out_cap: u64,
                            padding: *mut u32, chunk_len: *mut u32) -> c_int;
    pub fn chip_zfec_decode(k: u32, m: u32, input: *const u8, len: u64, padding: u32, out: *mut u8, out_cap: u64,
                            out_len: *mut u64) -> c_int;
    pub fn chip_zfec_decode_shares(k: u32, m: u32, shares: *const *const u8, idx: *const u32, nshares: u32,
                                   chunk_len: u64, padding: u32, out: *mut u8, out_cap: u64, out_len: *mut u64)
        -> c_int;
    pub fn chip_bao_encode(input: *const u8, n: u64, out: *mut u8, out_cap: u64, out_len: *mut u64,
                           hash: *mut u8) -> c_int;
    pub fn chip_bao_decode(enc: *const u8, len: u64, hash: *const u8, hash_len: u64, out: *mut u8, out_cap: u64,
                           out_len: *mut u64) -> c_int;
    pub fn chip_blake3(input: *const u8, n: u64, hash: *mut u8) -> c_int;

    // ---- host stages (host threads, no device)
    pub fn chip_snap_compress(input: *const u8, n: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_snap_decompress(input: *const u8, n: u64, out: *mut u8, out_cap: u64, out_len: *mut u64)
        -> c_int;
    pub fn chip_ecies_encrypt(pubkey: *const u8, pubkey_len: u64, inject: *const chip_ecies_inject,
                              input: *const u8, n: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_ecies_decrypt(secret_key: *const u8, sk_len: u64, input: *const u8, n: u64, out: *mut u8,
                              out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_ecies_public_key(secret_key: *const u8, pubkey: *mut u8) -> c_int;

    // ---- pipeline glue (host buffers)
    pub fn chip_encode(format: u8, pubkey: *const u8, pubkey_len: u64, inject: *const chip_ecies_inject,
                       input: *const u8, n: u64, out: *mut u8, out_cap: u64, out_len: *mut u64, hash: *mut u8,
                       info: *mut chip_encode_info) -> c_int;
    pub fn chip_decode(secret_key: *const u8, sk_len: u64, hash: *const u8, hash_len: u64, input: *const u8,
                       n: u64, padding: u32, format: u8, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;

    // ---- device-resident batch API (the throughput path)
    pub fn chip_zfec_encode_batch_dev(k: u32, m: u32, d_in: *const u8, in_stride: u64, n: u64, count: u64,
                                      d_out: *mut u8, out_stride: u64, stream: *mut c_void) -> c_int;
    pub fn chip_hbm_pattern_batch_dev(k: u32, m: u32, d_in: *const u8, in_stride: u64, n: u64, count: u64,
                                      d_out: *mut u8, out_stride: u64, stream: *mut c_void) -> c_int;
    pub fn chip_zfec_decode_batch_dev(k: u32, m: u32, d_in: *const u8, in_stride: u64, chunk_len: u64,
                                      idx: *const u32, nshares: u32, count: u64, d_out: *mut u8,
                                      out_stride: u64, stream: *mut c_void) -> c_int;
    pub fn chip_bao_scratch_len(n: u64, count: u64) -> u64;
    pub fn chip_bao_encode_batch_dev(d_in: *const u8, in_stride: u64, n: u64, count: u64, d_out: *mut u8,
                                     out_stride: u64, d_hash: *mut u8, d_scratch: *mut c_void,
                                     stream: *mut c_void) -> c_int;
    pub fn chip_bao_decode_batch_dev(d_in: *const u8, in_stride: u64, n: u64, count: u64, d_hash: *const u8,
                                     d_out: *mut u8, out_stride: u64, d_status: *mut u32, d_scratch: *mut c_void,
                                     stream: *mut c_void) -> c_int;
    pub fn chip_encode_scratch_len(format: u8, n: u64, count: u64) -> u64;
    pub fn chip_encode_batch_dev(format: u8, d_in: *const u8, in_stride: u64, n: u64, count: u64, d_out: *mut u8,
                                 out_stride: u64, out_len: *mut u64, d_hash: *mut u8, info: *mut chip_encode_info,
                                 d_scratch: *mut c_void, stream: *mut c_void) -> c_int;
    pub fn chip_decode_scratch_len(format: u8, in_len: u64, count: u64) -> u64;
    pub fn chip_decode_batch_dev(format: u8, d_in: *const u8, in_stride: u64, in_len: u64, count: u64,
                                 d_hash: *const u8, padding: u32, d_out: *mut u8, out_stride: u64,
                                 out_len: *mut u64, d_status: *mut u32, d_scratch: *mut c_void,
                                 stream: *mut c_void) -> c_int;

    // ---- slices and scrub (decoding.rs:116-212)
    pub fn chip_bao_slice_len(content_len: u64, start: u64, len: u64) -> u64;
    pub fn chip_bao_extract_slice(enc: *const u8, len: u64, index: u64, slice_len: u64, out: *mut u8,
                                  out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_bao_verify_slice(hash: *const u8, hash_len: u64, enc: *const u8, len: u64, index: u64,
                                 count: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_scrub(enc: *const u8, len: u64, hash: *const u8, hash_len: u64, padding: u32, chunk_len: u32,
                      out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn chip_scrub_scratch_len(len: u64, count: u64) -> u64;
    pub fn chip_scrub_batch_dev(d_in: *const u8, in_stride: u64, len: u64, count: u64, d_hash: *const u8,
                                padding: u32, chunk_len: u32, d_out: *mut u8, out_stride: u64, status: *mut i32,
                                d_scratch: *mut c_void, stream: *mut c_void) -> c_int;

    // ---- streaming bao hasher (utils.rs:104-137)
    pub fn chip_bao_hasher_new(out: *mut *mut chip_bao_hasher) -> c_int;
    pub fn chip_bao_hasher_update(h: *mut chip_bao_hasher, buf: *const u8, n: u64) -> c_int;
    pub fn chip_bao_hasher_finalize(h: *mut chip_bao_hasher, hash: *mut u8) -> c_int;
    pub fn chip_bao_hasher_len(h: *mut chip_bao_hasher) -> u64;
    pub fn chip_bao_hasher_read_all(h: *mut chip_bao_hasher, out: *mut u8, out_cap: u64, out_len: *mut u64)
        -> c_int;
    pub fn chip_bao_hasher_free(h: *mut chip_bao_hasher);
    pub fn chip_bao_hasher_drop_cache() -> u64;
    pub fn chip_bao_hasher_cached_bytes() -> u64;

    // ---- host-memory batch (host -> HBM -> host)
    pub fn chip_encode_host_batch(format: u8, pubkey: *const u8, pubkey_len: u64, inject: *const chip_ecies_inject,
                                  input: *const u8, n: u64, count: u64, in_stride: u64, out: *mut u8,
                                  out_stride: u64, out_len: *mut u64, hashes: *mut u8, info: *mut chip_encode_info,
                                  nslots: u32, slice_bytes: u64, host_threads: u32) -> c_int;
    pub fn chip_decode_host_batch(format: u8, secret_key: *const u8, sk_len: u64, hashes: *const u8,
                                  input: *const u8, in_len: *const u64, count: u64, in_stride: u64,
                                  padding: *const u32, out: *mut u8, out_stride: u64, out_len: *mut u64,
                                  status: *mut i32, nslots: u32, slice_bytes: u64, host_threads: u32) -> c_int;
}
