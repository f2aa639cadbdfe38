//! carbonado-hip: the MI355X (gfx950) hot path of carbonado's encode()/decode()
//! behind safe Rust wrappers over `libcarbonado_hip.so` (`include/carbonado_hip.h`).
//!
//! * Stage functions, one per crate-internal seam of carbonado 0.6.0
//!   (SURVEY.md §8b): [`zfec_encode`] <- `encoding::zfec` (encoding.rs:48),
//!   [`bao_encode`] <- `encoding::bao` (encoding.rs:39), [`zfec_decode`] <-
//!   `decoding::zfec` (decoding.rs:35), [`zfec_decode_shares`] <-
//!   `decoding::zfec_chunks` (decoding.rs:21), [`bao_decode`] <- `decoding::bao`
//!   (decoding.rs:54).  Inputs are borrowed slices, outputs fresh `Vec<u8>`s, as
//!   in the crate; the library copies pageable memory through its own pinned
//!   ring, so nothing needs registering.
//! * The glue ([`encode`], [`decode`]), slices and scrub, the host stages,
//!   the flat-file header and the streaming [`BaoHasher`].
//! * The device-resident batch API (the throughput path the benchmark is
//!   measured on): [`DeviceRows`] allocates through `chip_device_alloc`, the
//!   library's class-balanced HBM allocator (the 4-of-8 encode
//!   runs at 0.77 of the HBM roofline over it, 0.64 over a plain hipMalloc),
//!   so Rust callers get the fast placement by default; caller-owned device
//!   memory can be wrapped with [`DeviceRows::from_raw`].
//!
//! There is no CPU fallback: with no gfx950 device every compute call returns
//! [`ChipError::NoDevice`].
pub mod ffi;

use std::ffi::CStr;
use std::os::raw::{c_int, c_void};
use std::ptr;
use std::sync::OnceLock;

pub use ffi::chip_encode_info as ChipEncodeInfo;
pub use ffi::chip_header as ChipHeader;

pub const HASH_LEN: usize = ffi::CHIP_HASH_LEN;

/// One variant per `chip_status` (include/carbonado_hip.h), named after the
/// `CarbonadoError` variant it stands for (error.rs:7-115).
#[derive(Debug, Clone, PartialEq, Eq, thiserror::Error)]
pub enum ChipError {
    #[error("invalid argument")]
    InvalidArgument,
    #[error("output buffer too small: {0} bytes needed")]
    BufferTooSmall(u64),
    #[error("Input bytes must divide evenly over number of zfec chunks.")]
    UnevenZfecChunks,
    #[error("Hash must be 32 bytes long, an input of {0} bytes was provided.")]
    HashDecode(usize),
    #[error("bao decode: hash mismatch")]
    BaoHashMismatch,
    #[error("bao decode: truncated stream")]
    BaoTruncated,
    #[error("zfec: fewer than k distinct shares")]
    Zfec,
    #[error("Padding from Zfec should always be zero, since Carbonado adds its own padding.")]
    EncodeZfecPadding,
    #[error("Chunk length should be as calculated.")]
    EncodeInvalidChunkLength,
    #[error("Verifiable slice count should be evenly divisible by 8.")]
    InvalidVerifiableSliceCount,
    #[error("unsupported format bits")]
    UnsupportedFormat,
    #[error("Data does not need to be scrubbed.")]
    UnnecessaryScrub,
    #[error("Scrubbed padding should remain the same.")]
    ScrubbedPaddingMismatch,
    #[error("Mismatch between scrubbed data length and input length.")]
    ScrubbedLengthMismatch,
    #[error("Scrubbed hash is not equal to original hash.")]
    InvalidScrubbedHash,
    #[error("snappy framing error")]
    Snap,
    #[error("ecies error (bad key or tag)")]
    Ecies,
    #[error("secp256k1 error")]
    Secp256k1,
    #[error("Invalid header length calculation")]
    InvalidHeaderLength,
    #[error("File header lacks Carbonado magic number.")]
    InvalidMagic,
    #[error("no usable gfx950 device: {0}")]
    NoDevice(String),
    #[error("HIP runtime error: {0}")]
    Device(String),
    #[error("libcarbonado_hip has ABI {0}, this crate binds ABI {abi}", abi = ffi::CHIP_ABI_VERSION)]
    AbiMismatch(i32),
    #[error("status {0}: {1}")]
    Other(i32, String),
}

fn cstr(p: *const std::os::raw::c_char) -> String {
    if p.is_null() {
        return String::new();
    }
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

impl ChipError {
    /// The error for a non-zero status.  `hash_len` fills HashDecode,
    /// `needed` BufferTooSmall (the size the call reported in *out_len).
    pub fn from_status(rc: c_int, hash_len: usize, needed: u64) -> ChipError {
        match rc {
            ffi::CHIP_ERR_INVALID_ARG => ChipError::InvalidArgument,
            ffi::CHIP_ERR_BUFFER_TOO_SMALL => ChipError::BufferTooSmall(needed),
            ffi::CHIP_ERR_UNEVEN_ZFEC_CHUNKS => ChipError::UnevenZfecChunks,
            ffi::CHIP_ERR_HASH_DECODE => ChipError::HashDecode(hash_len),
            ffi::CHIP_ERR_BAO_HASH_MISMATCH => ChipError::BaoHashMismatch,
            ffi::CHIP_ERR_BAO_TRUNCATED => ChipError::BaoTruncated,
            ffi::CHIP_ERR_ZFEC => ChipError::Zfec,
            ffi::CHIP_ERR_ENCODE_ZFEC_PADDING => ChipError::EncodeZfecPadding,
            ffi::CHIP_ERR_ENCODE_INVALID_CHUNK_LENGTH => ChipError::EncodeInvalidChunkLength,
            ffi::CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT => ChipError::InvalidVerifiableSliceCount,
            ffi::CHIP_ERR_UNSUPPORTED_FORMAT => ChipError::UnsupportedFormat,
            ffi::CHIP_ERR_UNNECESSARY_SCRUB => ChipError::UnnecessaryScrub,
            ffi::CHIP_ERR_SCRUBBED_PADDING_MISMATCH => ChipError::ScrubbedPaddingMismatch,
            ffi::CHIP_ERR_SCRUBBED_LENGTH_MISMATCH => ChipError::ScrubbedLengthMismatch,
            ffi::CHIP_ERR_INVALID_SCRUBBED_HASH => ChipError::InvalidScrubbedHash,
            ffi::CHIP_ERR_SNAP => ChipError::Snap,
            ffi::CHIP_ERR_ECIES => ChipError::Ecies,
            ffi::CHIP_ERR_SECP256K1 => ChipError::Secp256k1,
            ffi::CHIP_ERR_INVALID_HEADER_LENGTH => ChipError::InvalidHeaderLength,
            ffi::CHIP_ERR_INVALID_MAGIC => ChipError::InvalidMagic,
            ffi::CHIP_ERR_NO_DEVICE => ChipError::NoDevice(cstr(unsafe { ffi::chip_last_device_error() })),
            ffi::CHIP_ERR_DEVICE => ChipError::Device(cstr(unsafe { ffi::chip_last_device_error() })),
            s => ChipError::Other(s, cstr(unsafe { ffi::chip_strerror(s) })),
        }
    }

    /// The `chip_status` this error came from (for per-object status arrays).
    pub fn status(&self) -> c_int {
        match self {
            ChipError::InvalidArgument => ffi::CHIP_ERR_INVALID_ARG,
            ChipError::BufferTooSmall(_) => ffi::CHIP_ERR_BUFFER_TOO_SMALL,
            ChipError::UnevenZfecChunks => ffi::CHIP_ERR_UNEVEN_ZFEC_CHUNKS,
            ChipError::HashDecode(_) => ffi::CHIP_ERR_HASH_DECODE,
            ChipError::BaoHashMismatch => ffi::CHIP_ERR_BAO_HASH_MISMATCH,
            ChipError::BaoTruncated => ffi::CHIP_ERR_BAO_TRUNCATED,
            ChipError::Zfec => ffi::CHIP_ERR_ZFEC,
            ChipError::EncodeZfecPadding => ffi::CHIP_ERR_ENCODE_ZFEC_PADDING,
            ChipError::EncodeInvalidChunkLength => ffi::CHIP_ERR_ENCODE_INVALID_CHUNK_LENGTH,
            ChipError::InvalidVerifiableSliceCount => ffi::CHIP_ERR_INVALID_VERIFIABLE_SLICE_COUNT,
            ChipError::UnsupportedFormat => ffi::CHIP_ERR_UNSUPPORTED_FORMAT,
            ChipError::UnnecessaryScrub => ffi::CHIP_ERR_UNNECESSARY_SCRUB,
            ChipError::ScrubbedPaddingMismatch => ffi::CHIP_ERR_SCRUBBED_PADDING_MISMATCH,
            ChipError::ScrubbedLengthMismatch => ffi::CHIP_ERR_SCRUBBED_LENGTH_MISMATCH,
            ChipError::InvalidScrubbedHash => ffi::CHIP_ERR_INVALID_SCRUBBED_HASH,
            ChipError::Snap => ffi::CHIP_ERR_SNAP,
            ChipError::Ecies => ffi::CHIP_ERR_ECIES,
            ChipError::Secp256k1 => ffi::CHIP_ERR_SECP256K1,
            ChipError::InvalidHeaderLength => ffi::CHIP_ERR_INVALID_HEADER_LENGTH,
            ChipError::InvalidMagic => ffi::CHIP_ERR_INVALID_MAGIC,
            ChipError::NoDevice(_) => ffi::CHIP_ERR_NO_DEVICE,
            ChipError::Device(_) | ChipError::AbiMismatch(_) => ffi::CHIP_ERR_DEVICE,
            ChipError::Other(s, _) => *s,
        }
    }
}

pub type Result<T> = std::result::Result<T, ChipError>;

fn check(rc: c_int) -> Result<()> {
    if rc == ffi::CHIP_OK {
        Ok(())
    } else {
        Err(ChipError::from_status(rc, 0, 0))
    }
}

/// The loaded library must speak the ABI these declarations were written for.
fn abi() -> Result<()> {
    static ABI: OnceLock<c_int> = OnceLock::new();
    let v = *ABI.get_or_init(|| unsafe { ffi::chip_abi_version() });
    if v == ffi::CHIP_ABI_VERSION {
        Ok(())
    } else {
        Err(ChipError::AbiMismatch(v))
    }
}

/// Select the process's GPU (one process per GPU; idempotent).  Without it
/// the library follows the calling thread's current HIP device.
pub fn init(device: i32) -> Result<()> {
    abi()?;
    check(unsafe { ffi::chip_init(device) })
}

/// Run `f(out_ptr, cap, &mut out_len)` into a fresh Vec of capacity `cap`.
fn into_vec(cap: usize, hash_len: usize, f: impl FnOnce(*mut u8, u64, &mut u64) -> c_int) -> Result<Vec<u8>> {
    abi()?;
    let mut out: Vec<u8> = Vec::with_capacity(cap);
    let mut len = 0u64;
    let rc = f(out.as_mut_ptr(), cap as u64, &mut len);
    if rc != ffi::CHIP_OK {
        return Err(ChipError::from_status(rc, hash_len, len));
    }
    assert!(len as usize <= cap, "library reported {len} bytes into a {cap}-byte buffer");
    unsafe { out.set_len(len as usize) };
    Ok(out)
}

/// `into_vec`, retried once with the size a BUFFER_TOO_SMALL reported
/// (snappy output sizes are only known after decompression).
fn into_vec_grow(cap: usize, hash_len: usize, f: impl Fn(*mut u8, u64, &mut u64) -> c_int) -> Result<Vec<u8>> {
    match into_vec(cap, hash_len, &f) {
        Err(ChipError::BufferTooSmall(need)) if need as usize > cap => into_vec(need as usize, hash_len, &f),
        r => r,
    }
}

// ---- size helpers (utils.rs:47-58, bao's encoded_size) --------------------

/// utils::calc_padding_len with FEC_K generalised to k: (padding, chunk_len).
pub fn calc_padding_len(input_len: usize, k: u32) -> Result<(u32, u32)> {
    let (mut pad, mut chunk) = (0u32, 0u32);
    check(unsafe { ffi::chip_calc_padding_len(input_len as u64, k, &mut pad, &mut chunk) })?;
    Ok((pad, chunk))
}

pub fn zfec_encoded_len(input_len: usize, k: u32, m: u32) -> usize {
    unsafe { ffi::chip_zfec_encoded_len(input_len as u64, k, m) as usize }
}

pub fn bao_encoded_len(content_len: usize) -> usize {
    unsafe { ffi::chip_bao_encoded_len(content_len as u64) as usize }
}

pub fn encode_max_len(input_len: usize) -> usize {
    unsafe { ffi::chip_encode_max_len(input_len as u64) as usize }
}

// ---- the five seam functions -------------------------------------------------

/// encoding::zfec (encoding.rs:48-81): (shards [S0|..|S(m-1)], padding, chunk_len).
pub fn zfec_encode(input: &[u8], k: u32, m: u32) -> Result<(Vec<u8>, u32, u32)> {
    abi()?;
    let total = zfec_encoded_len(input.len(), k, m);
    let mut out: Vec<u8> = Vec::with_capacity(total);
    let (mut pad, mut chunk) = (0u32, 0u32);
    check(unsafe {
        ffi::chip_zfec_encode(k, m, input.as_ptr(), input.len() as u64, out.as_mut_ptr(), total as u64, &mut pad,
                              &mut chunk)
    })?;
    unsafe { out.set_len(total) };
    Ok((out, pad, chunk))
}

/// decoding::zfec (decoding.rs:35-51): shards indexed by position, as the crate does.
pub fn zfec_decode(input: &[u8], padding: u32, k: u32, m: u32) -> Result<Vec<u8>> {
    let cap = if m == 0 { 0 } else { input.len() / m as usize * k as usize };
    into_vec(cap, 0, |out, cap, len| unsafe {
        ffi::chip_zfec_decode(k, m, input.as_ptr(), input.len() as u64, padding, out, cap, len)
    })
}

/// decoding::zfec_chunks (decoding.rs:21-32) with explicit share indices
/// (`decoding::zfec_chunks` passes 0..n, the crate's positional numbering).
pub fn zfec_decode_shares(shares: &[&[u8]], idx: &[u32], padding: u32, k: u32, m: u32) -> Result<Vec<u8>> {
    if shares.len() != idx.len() {
        return Err(ChipError::InvalidArgument);
    }
    let chunk = shares.first().map_or(0, |s| s.len());
    if shares.iter().any(|s| s.len() != chunk) {
        return Err(ChipError::InvalidArgument);
    }
    let ptrs: Vec<*const u8> = shares.iter().map(|s| s.as_ptr()).collect();
    into_vec(k as usize * chunk, 0, |out, cap, len| unsafe {
        ffi::chip_zfec_decode_shares(k, m, ptrs.as_ptr(), idx.as_ptr(), shares.len() as u32, chunk as u64, padding,
                                     out, cap, len)
    })
}

/// encoding::bao (encoding.rs:38-44): the combined pre-order stream and its root hash.
pub fn bao_encode(input: &[u8]) -> Result<(Vec<u8>, [u8; HASH_LEN])> {
    let mut hash = [0u8; HASH_LEN];
    let enc = into_vec(bao_encoded_len(input.len()), 0, |out, cap, len| unsafe {
        ffi::chip_bao_encode(input.as_ptr(), input.len() as u64, out, cap, len, hash.as_mut_ptr())
    })?;
    Ok((enc, hash))
}

/// decoding::bao (decoding.rs:53-60): every node verified, the content returned.
pub fn bao_decode(input: &[u8], hash: &[u8]) -> Result<Vec<u8>> {
    into_vec(input.len(), hash.len(), |out, cap, len| unsafe {
        ffi::chip_bao_decode(input.as_ptr(), input.len() as u64, hash.as_ptr(), hash.len() as u64, out, cap, len)
    })
}

/// BLAKE3 of `input` (== the bao root hash), computed on the device.
pub fn blake3(input: &[u8]) -> Result<[u8; HASH_LEN]> {
    abi()?;
    let mut hash = [0u8; HASH_LEN];
    check(unsafe { ffi::chip_blake3(input.as_ptr(), input.len() as u64, hash.as_mut_ptr()) })?;
    Ok(hash)
}

// ---- slices and scrub (decoding.rs:116-212) -------------------------------

/// extract_slice (decoding.rs:116-127) with a u64 index (the crate's u16
/// `index * SLICE_LEN` wraps at index 64).
pub fn extract_slice(encoded: &[u8], index: u64) -> Result<Vec<u8>> {
    let content = encoded_content_len(encoded)?;
    let cap = unsafe { ffi::chip_bao_slice_len(content, index * ffi::CHIP_SLICE_LEN as u64, ffi::CHIP_SLICE_LEN as u64) };
    into_vec(cap as usize, 0, |out, cap, len| unsafe {
        ffi::chip_bao_extract_slice(encoded.as_ptr(), encoded.len() as u64, index, ffi::CHIP_SLICE_LEN as u64, out,
                                    cap, len)
    })
}

/// verify_slice (decoding.rs:129-149): `count` 1 KiB slices from `index`, verified.
pub fn verify_slice(hash: &[u8], input: &[u8], index: u64, count: u64) -> Result<Vec<u8>> {
    let cap = (count as usize).saturating_mul(ffi::CHIP_SLICE_LEN).min(input.len());
    into_vec(cap, hash.len(), |out, cap, len| unsafe {
        ffi::chip_bao_verify_slice(hash.as_ptr(), hash.len() as u64, input.as_ptr(), input.len() as u64, index, count,
                                   out, cap, len)
    })
}

/// scrub (decoding.rs:151-212), decoding the good shards with their TRUE
/// indices.  An intact stream is `Err(ChipError::UnnecessaryScrub)`.
pub fn scrub(input: &[u8], hash: &[u8], padding: u32, chunk_len: u32) -> Result<Vec<u8>> {
    into_vec(input.len(), hash.len(), |out, cap, len| unsafe {
        ffi::chip_scrub(input.as_ptr(), input.len() as u64, hash.as_ptr(), hash.len() as u64, padding, chunk_len,
                        out, cap, len)
    })
}

fn encoded_content_len(encoded: &[u8]) -> Result<u64> {
    let head: [u8; 8] = encoded.get(..8).and_then(|h| h.try_into().ok()).ok_or(ChipError::BaoTruncated)?;
    Ok(u64::from_le_bytes(head))
}

// ---- host stages (encoding.rs:16-36, decoding.rs:62-77) ---------------------

/// The two values ecies::encrypt draws from thread_rng, for bit-exact tests;
/// production code passes `None` (fresh random values, as the crate).
#[derive(Clone, Copy, Debug)]
pub struct EciesInject<'a> {
    pub ephemeral_sk: &'a [u8; 32],
    pub nonce: &'a [u8; 16],
}

fn inject_ptr(inject: Option<EciesInject<'_>>, slot: &mut ffi::chip_ecies_inject) -> *const ffi::chip_ecies_inject {
    match inject {
        None => ptr::null(),
        Some(i) => {
            *slot = ffi::chip_ecies_inject { ephemeral_sk: i.ephemeral_sk.as_ptr(), nonce: i.nonce.as_ptr() };
            slot
        }
    }
}

pub fn snap_compress(input: &[u8]) -> Result<Vec<u8>> {
    let cap = unsafe { ffi::chip_snap_max_len(input.len() as u64) } as usize;
    into_vec(cap, 0, |out, cap, len| unsafe {
        ffi::chip_snap_compress(input.as_ptr(), input.len() as u64, out, cap, len)
    })
}

pub fn snap_decompress(input: &[u8]) -> Result<Vec<u8>> {
    into_vec_grow(input.len().saturating_mul(2).max(1024), 0, |out, cap, len| unsafe {
        ffi::chip_snap_decompress(input.as_ptr(), input.len() as u64, out, cap, len)
    })
}

pub fn ecies_encrypt(pubkey: &[u8], input: &[u8], inject: Option<EciesInject<'_>>) -> Result<Vec<u8>> {
    let mut slot = ffi::chip_ecies_inject { ephemeral_sk: ptr::null(), nonce: ptr::null() };
    let inj = inject_ptr(inject, &mut slot);
    into_vec(input.len() + 97, 0, |out, cap, len| unsafe {
        ffi::chip_ecies_encrypt(pubkey.as_ptr(), pubkey.len() as u64, inj, input.as_ptr(), input.len() as u64, out,
                                cap, len)
    })
}

pub fn ecies_decrypt(input: &[u8], secret_key: &[u8]) -> Result<Vec<u8>> {
    into_vec(input.len(), 0, |out, cap, len| unsafe {
        ffi::chip_ecies_decrypt(secret_key.as_ptr(), secret_key.len() as u64, input.as_ptr(), input.len() as u64,
                                out, cap, len)
    })
}

// ---- encode() / decode() glue (encoding.rs:86-172, decoding.rs:80-114) ------

/// encoding::encode: (stream, hash, EncodeInfo), the crate's `Encoded`.
pub fn encode(pubkey: &[u8], input: &[u8], format: u8, inject: Option<EciesInject<'_>>)
              -> Result<(Vec<u8>, [u8; HASH_LEN], ChipEncodeInfo)> {
    let mut hash = [0u8; HASH_LEN];
    let mut info = ChipEncodeInfo::default();
    let mut slot = ffi::chip_ecies_inject { ephemeral_sk: ptr::null(), nonce: ptr::null() };
    let inj = inject_ptr(inject, &mut slot);
    let out = into_vec(encode_max_len(input.len()), 0, |out, cap, len| unsafe {
        ffi::chip_encode(format, pubkey.as_ptr(), pubkey.len() as u64, inj, input.as_ptr(), input.len() as u64, out,
                         cap, len, hash.as_mut_ptr(), &mut info)
    })?;
    Ok((out, hash, info))
}

/// decoding::decode: bao -> zfec on the device, ecies -> snap on the host.
pub fn decode(secret_key: &[u8], hash: &[u8], input: &[u8], padding: u32, format: u8) -> Result<Vec<u8>> {
    into_vec_grow(input.len().max(1024), hash.len(), |out, cap, len| unsafe {
        ffi::chip_decode(secret_key.as_ptr(), secret_key.len() as u64, hash.as_ptr(), hash.len() as u64,
                         input.as_ptr(), input.len() as u64, padding, format, out, cap, len)
    })
}

// ---- flat-file container (file.rs) ---------------------------------------

/// Header::new (file.rs:263-289).  `aux` = the signature's auxiliary
/// randomness (None = fresh, as the crate).
#[allow(clippy::too_many_arguments)]
pub fn header_new(sk: &[u8], pk: &[u8], hash: &[u8], format: u8, chunk_index: u8, encoded_len: u32,
                  padding_len: u32, metadata: Option<&[u8; 8]>, aux: Option<&[u8; 32]>) -> Result<ChipHeader> {
    abi()?;
    let mut h = ChipHeader::default();
    check(unsafe {
        ffi::chip_header_new(sk.as_ptr(), sk.len() as u64, pk.as_ptr(), pk.len() as u64, hash.as_ptr(),
                             hash.len() as u64, format, chunk_index, encoded_len, padding_len,
                             metadata.map_or(ptr::null(), |m| m.as_ptr()), aux.map_or(ptr::null(), |a| a.as_ptr()),
                             &mut h)
    })?;
    Ok(h)
}

/// Header::try_to_vec (file.rs:292-335).
pub fn header_to_bytes(h: &ChipHeader) -> Result<[u8; ffi::CHIP_HEADER_LEN]> {
    let mut out = [0u8; ffi::CHIP_HEADER_LEN];
    check(unsafe { ffi::chip_header_to_bytes(h, out.as_mut_ptr()) })?;
    Ok(out)
}

/// Header::try_from(&[u8]) (file.rs:116-154); a short slice is an error, not a panic.
pub fn header_parse(bytes: &[u8]) -> Result<ChipHeader> {
    let mut h = ChipHeader::default();
    check(unsafe { ffi::chip_header_parse(bytes.as_ptr(), bytes.len() as u64, &mut h) })?;
    Ok(h)
}

/// file::encode (file.rs:409-440): header || encode(pubkey, input, level).
pub fn file_encode(sk: &[u8], pk: Option<&[u8]>, input: &[u8], level: u8, metadata: Option<&[u8; 8]>)
                   -> Result<(Vec<u8>, ChipEncodeInfo)> {
    let mut info = ChipEncodeInfo::default();
    let (pkp, pkl) = pk.map_or((ptr::null(), 0u64), |p| (p.as_ptr(), p.len() as u64));
    let out = into_vec(ffi::CHIP_HEADER_LEN + encode_max_len(input.len()), 0, |out, cap, len| unsafe {
        ffi::chip_file_encode(sk.as_ptr(), sk.len() as u64, pkp, pkl, input.as_ptr(), input.len() as u64, level,
                              metadata.map_or(ptr::null(), |m| m.as_ptr()), ptr::null(), ptr::null(), out, cap, len,
                              &mut info)
    })?;
    Ok((out, info))
}

/// file::decode (file.rs:395-407): (header, decoded content).
pub fn file_decode(sk: &[u8], input: &[u8]) -> Result<(ChipHeader, Vec<u8>)> {
    let mut hdr = ChipHeader::default();
    let hdrp: *mut ChipHeader = &mut hdr; // the retry closure must be Fn
    let out = into_vec_grow(input.len().max(1024), 0, |out, cap, len| unsafe {
        ffi::chip_file_decode(sk.as_ptr(), sk.len() as u64, input.as_ptr(), input.len() as u64, hdrp, out, cap, len)
    })?;
    Ok((hdr, out))
}

// ---- streaming hasher (utils.rs:104-137) ----------------------------------

/// utils::BaoHasher: appends land in HBM, chunk CVs are hashed as whole
/// units arrive; `finalize` lays the stream out and builds the parents.
pub struct BaoHasher(*mut ffi::chip_bao_hasher);

// the library serialises every call on one hasher with its own mutex
unsafe impl Send for BaoHasher {}
unsafe impl Sync for BaoHasher {}

impl BaoHasher {
    pub fn new() -> Result<BaoHasher> {
        abi()?;
        let mut h = ptr::null_mut();
        check(unsafe { ffi::chip_bao_hasher_new(&mut h) })?;
        Ok(BaoHasher(h))
    }

    /// The bytes are copied before this returns.
    pub fn update(&self, buf: &[u8]) -> Result<()> {
        check(unsafe { ffi::chip_bao_hasher_update(self.0, buf.as_ptr(), buf.len() as u64) })
    }

    pub fn finalize(&self) -> Result<[u8; HASH_LEN]> {
        let mut hash = [0u8; HASH_LEN];
        check(unsafe { ffi::chip_bao_hasher_finalize(self.0, hash.as_mut_ptr()) })?;
        Ok(hash)
    }

    pub fn len(&self) -> u64 {
        unsafe { ffi::chip_bao_hasher_len(self.0) }
    }

    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// The combined bao encoding (after `finalize`).
    pub fn read_all(&self) -> Result<Vec<u8>> {
        let cap = bao_encoded_len(self.len() as usize);
        into_vec(cap, 0, |out, cap, len| unsafe { ffi::chip_bao_hasher_read_all(self.0, out, cap, len) })
    }
}

impl Drop for BaoHasher {
    fn drop(&mut self) {
        unsafe { ffi::chip_bao_hasher_free(self.0) }
    }
}

/// Destroy every parked (freed, kept for reuse) hasher; returns the device
/// bytes freed.  Parked hashers hold at most CHIP_HASHER_PARK_MIB (3 GiB).
pub fn drop_hasher_cache() -> u64 {
    unsafe { ffi::chip_bao_hasher_drop_cache() }
}

/// Device bytes the parked hashers hold.
pub fn hasher_cached_bytes() -> u64 {
    unsafe { ffi::chip_bao_hasher_cached_bytes() }
}

/// Where this process's host-copy path sits on the box (JSON): the GPU's
/// NUMA node, the staging ring's node, the copy workers' nodes (diagnostic).
pub fn host_topology() -> Result<String> {
    abi()?;
    let mut len = 0u64;
    let _ = unsafe { ffi::chip_host_topology(ptr::null_mut(), 0, &mut len) };
    let mut buf = vec![0u8; len.max(1) as usize];
    check(unsafe { ffi::chip_host_topology(buf.as_mut_ptr() as *mut std::os::raw::c_char, len, &mut len) })?;
    buf.truncate(len.saturating_sub(1) as usize);
    Ok(String::from_utf8_lossy(&buf).into_owned())
}

// ---- device-resident batch API ----------------------------------------------

/// A HIP stream handle (`hipStream_t`); [`Stream::DEFAULT`] = the library's
/// per-thread stream.  The batch calls enqueue on it and return.  The handle
/// is private: safe code gets only [`Stream::DEFAULT`]; a caller's own stream
/// comes in through [`Stream::from_raw`], whose caller vouches for it.
#[derive(Clone, Copy, Debug)]
pub struct Stream(*mut c_void);

impl Stream {
    pub const DEFAULT: Stream = Stream(ptr::null_mut());

    /// # Safety
    /// `raw` must be a live `hipStream_t` of the device the library runs on,
    /// and stay alive until the work enqueued on it through this handle has
    /// finished.
    pub unsafe fn from_raw(raw: *mut c_void) -> Stream {
        Stream(raw)
    }

    pub fn as_raw(&self) -> *mut c_void {
        self.0
    }
}

unsafe impl Send for Stream {}
unsafe impl Sync for Stream {}

/// Device memory from `chip_device_alloc`: class-balanced from 1 GiB up
/// (DESIGN.md §2), contiguous below.  Freed on drop.
pub struct DeviceBuffer {
    ptr: *mut c_void,
    len: usize,
}

unsafe impl Send for DeviceBuffer {}
unsafe impl Sync for DeviceBuffer {}

impl DeviceBuffer {
    pub fn new(bytes: usize) -> Result<DeviceBuffer> {
        abi()?;
        let mut p = ptr::null_mut();
        check(unsafe { ffi::chip_device_alloc(bytes as u64, &mut p) })?;
        Ok(DeviceBuffer { ptr: p, len: bytes })
    }

    pub fn len(&self) -> usize {
        self.len
    }

    pub fn is_empty(&self) -> bool {
        self.len == 0
    }

    pub fn as_ptr(&self) -> *const u8 {
        self.ptr as *const u8
    }

    pub fn as_mut_ptr(&mut self) -> *mut u8 {
        self.ptr as *mut u8
    }

    /// (memory classes found, classes used, seconds) of a class-balanced buffer.
    pub fn alloc_info(&self) -> Result<(u32, u32, f64)> {
        let (mut f, mut u, mut s) = (0u32, 0u32, 0f64);
        check(unsafe { ffi::chip_device_alloc_info(self.ptr, &mut f, &mut u, &mut s) })?;
        Ok((f, u, s))
    }
}

impl Drop for DeviceBuffer {
    fn drop(&mut self) {
        if !self.ptr.is_null() {
            unsafe { ffi::chip_device_free(self.ptr) };
        }
    }
}

enum Mem {
    Owned(DeviceBuffer),
    Borrowed(*mut u8, usize),
}

/// `count` rows of `row` bytes at a 16-B multiple `stride` (256-B from `alloc`) in device memory:
/// the shape every batch entry point takes (object o at base + o * stride).
pub struct DeviceRows {
    mem: Mem,
    pub count: u64,
    pub row: u64,
    pub stride: u64,
    off: u64, // where row 0 starts in `mem` (alloc_streams: STREAM_OFFSET)
}

/// Where `DeviceRows::alloc_streams` puts each bao stream in its row: after
/// the stream's 8-byte header every chunk and parent node then starts on a
/// 64-B boundary, which runs level 12 4-11 % and decode 4-12 % faster than
/// streams at the row start.
pub const STREAM_OFFSET: u64 = 56;

unsafe impl Send for DeviceRows {}

impl DeviceRows {
    /// Allocate through `chip_device_alloc` (the default: the fast placement).
    pub fn alloc(count: u64, row: u64) -> Result<DeviceRows> {
        // 256-B pitch: every row's 128-B pieces start on a memory line (a 16-B pitch
        // costs the kernels 1.21x the read traffic)
        let stride = (row + 255) / 256 * 256;
        let buf = DeviceBuffer::new((count * stride).max(16) as usize)?;
        Ok(DeviceRows { mem: Mem::Owned(buf), count, row, stride, off: 0 })
    }

    /// Rows for the bao streams of `content_len`-byte contents (the output of
    /// `encode_batch` at Zfec|Bao with content 8 * chunk_len, or of
    /// `bao_encode_batch`), each stream STREAM_OFFSET bytes into its row when
    /// it has more than 512 chunks (the entry points take those at any 8-B
    /// phase; smaller streams stay at the row start).
    pub fn alloc_streams(count: u64, content_len: u64) -> Result<DeviceRows> {
        let len = bao_encoded_len(content_len as usize) as u64;
        let off = if content_len > 512 * 1024 { STREAM_OFFSET } else { 0 };
        let stride = (off + len + 255) / 256 * 256;
        let buf = DeviceBuffer::new((count * stride).max(16) as usize)?;
        Ok(DeviceRows { mem: Mem::Owned(buf), count, row: len, stride, off })
    }

    /// Wrap caller-owned device memory (any 16-B aligned allocation works,
    /// only slower than `alloc`'s).
    ///
    /// # Safety
    /// `base` must point to at least `(count - 1) * stride + row` bytes of
    /// device memory that outlive the returned value.
    pub unsafe fn from_raw(base: *mut u8, count: u64, row: u64, stride: u64) -> Result<DeviceRows> {
        if base as usize % 16 != 0 || stride % 16 != 0 || (count > 1 && stride < row) {
            return Err(ChipError::InvalidArgument);
        }
        let bytes = if count == 0 { 0 } else { ((count - 1) * stride + row) as usize };
        Ok(DeviceRows { mem: Mem::Borrowed(base, bytes), count, row, stride, off: 0 })
    }

    /// Bytes from row 0's start to the end of the memory.
    fn bytes(&self) -> usize {
        let total = match &self.mem {
            Mem::Owned(b) => b.len(),
            Mem::Borrowed(_, n) => *n,
        };
        total.saturating_sub(self.off as usize)
    }

    /// Row 0's first byte.
    pub fn as_ptr(&self) -> *const u8 {
        let base = match &self.mem {
            Mem::Owned(b) => b.as_ptr(),
            Mem::Borrowed(p, _) => *p as *const u8,
        };
        base.wrapping_add(self.off as usize)
    }

    pub fn as_mut_ptr(&mut self) -> *mut u8 {
        let off = self.off as usize;
        let base = match &mut self.mem {
            Mem::Owned(b) => b.as_mut_ptr(),
            Mem::Borrowed(p, _) => *p,
        };
        base.wrapping_add(off)
    }

    /// The rows hold `count` objects of at least `row` bytes each.
    fn holds(&self, count: u64, row: u64) -> Result<()> {
        let need = if count == 0 { 0 } else { (count - 1) * self.stride + row };
        if count > self.count || row > self.stride.max(self.row) || need as usize > self.bytes() {
            return Err(ChipError::InvalidArgument);
        }
        Ok(())
    }
}

/// Scratch of a batch call, sized by the matching `*_scratch_len`.
pub fn scratch(bytes: u64) -> Result<DeviceBuffer> {
    DeviceBuffer::new(bytes.max(16) as usize)
}

/// zfec k-of-m encode of `input.count` objects of `n` bytes (encoding.rs:48-81
/// per object): object o's m shards to row o of `out`.
pub fn zfec_encode_batch(k: u32, m: u32, input: &DeviceRows, n: u64, out: &mut DeviceRows, stream: Stream)
                         -> Result<()> {
    input.holds(input.count, n)?;
    out.holds(input.count, zfec_encoded_len(n as usize, k, m) as u64)?;
    check(unsafe {
        ffi::chip_zfec_encode_batch_dev(k, m, input.as_ptr(), input.stride, n, input.count, out.as_mut_ptr(),
                                        out.stride, stream.0)
    })
}

/// Erasure decode (decoding.rs:21-51 with true indices): `idx` names the
/// shares present in each row of `input` (shard i at i * chunk_len), the
/// k * chunk_len data bytes of object o go to row o of `out`.
pub fn zfec_decode_batch(k: u32, m: u32, input: &DeviceRows, chunk_len: u64, idx: &[u32], out: &mut DeviceRows,
                         stream: Stream) -> Result<()> {
    input.holds(input.count, m as u64 * chunk_len)?;
    out.holds(input.count, k as u64 * chunk_len)?;
    check(unsafe {
        ffi::chip_zfec_decode_batch_dev(k, m, input.as_ptr(), input.stride, chunk_len, idx.as_ptr(),
                                        idx.len() as u32, input.count, out.as_mut_ptr(), out.stride, stream.0)
    })
}

/// bao encode of every row (encoding.rs:38-44): streams to `out`, hashes to
/// `hashes` (count * 32 bytes).  `scratch`: [`bao_scratch_len`] bytes.
pub fn bao_encode_batch(input: &DeviceRows, n: u64, out: &mut DeviceRows, hashes: &mut DeviceBuffer,
                        scratch: &mut DeviceBuffer, stream: Stream) -> Result<()> {
    input.holds(input.count, n)?;
    out.holds(input.count, bao_encoded_len(n as usize) as u64)?;
    if hashes.len() < input.count as usize * HASH_LEN || (scratch.len() as u64) < bao_scratch_len(n, input.count) {
        return Err(ChipError::InvalidArgument);
    }
    check(unsafe {
        ffi::chip_bao_encode_batch_dev(input.as_ptr(), input.stride, n, input.count, out.as_mut_ptr(), out.stride,
                                       hashes.as_mut_ptr(), scratch.ptr, stream.0)
    })
}

pub fn bao_scratch_len(n: u64, count: u64) -> u64 {
    unsafe { ffi::chip_bao_scratch_len(n, count) }
}

/// bao verify-decode of every row (decoding.rs:53-60): content to `out`,
/// per-object status (u32, 0 or a chip_status) to `status` (count * 4 bytes).
pub fn bao_decode_batch(input: &DeviceRows, n: u64, hashes: &DeviceBuffer, out: &mut DeviceRows,
                        status: &mut DeviceBuffer, scratch: &mut DeviceBuffer, stream: Stream) -> Result<()> {
    input.holds(input.count, bao_encoded_len(n as usize) as u64)?;
    out.holds(input.count, n)?;
    if hashes.len() < input.count as usize * HASH_LEN || status.len() < input.count as usize * 4 ||
        (scratch.len() as u64) < bao_scratch_len(n, input.count) {
        return Err(ChipError::InvalidArgument);
    }
    check(unsafe {
        ffi::chip_bao_decode_batch_dev(input.as_ptr(), input.stride, n, input.count, hashes.as_ptr(),
                                       out.as_mut_ptr(), out.stride, status.as_mut_ptr() as *mut u32, scratch.ptr,
                                       stream.0)
    })
}

pub fn encode_scratch_len(format: u8, n: u64, count: u64) -> u64 {
    unsafe { ffi::chip_encode_scratch_len(format, n, count) }
}

pub fn decode_scratch_len(format: u8, in_len: u64, count: u64) -> u64 {
    unsafe { ffi::chip_decode_scratch_len(format, in_len, count) }
}

/// encode() (encoding.rs:86-172) of every row at a device-only level (Bao
/// and/or Zfec bits; Zfec|Bao runs fused).  Returns (encoded length, EncodeInfo).
pub fn encode_batch(format: u8, input: &DeviceRows, n: u64, out: &mut DeviceRows, hashes: &mut DeviceBuffer,
                    scratch: &mut DeviceBuffer, stream: Stream) -> Result<(u64, ChipEncodeInfo)> {
    input.holds(input.count, n)?;
    if hashes.len() < input.count as usize * HASH_LEN ||
        (scratch.len() as u64) < encode_scratch_len(format, n, input.count) {
        return Err(ChipError::InvalidArgument);
    }
    let mut out_len = 0u64;
    let mut info = ChipEncodeInfo::default();
    check(unsafe {
        ffi::chip_encode_batch_dev(format, input.as_ptr(), input.stride, n, input.count, out.as_mut_ptr(),
                                   out.stride, &mut out_len, hashes.as_mut_ptr(), &mut info, scratch.ptr, stream.0)
    })?;
    Ok((out_len, info))
}

/// decode() (decoding.rs:80-114) of every row at a device-only level; per-object
/// status (u32) to `status`.  Returns the decoded length.
#[allow(clippy::too_many_arguments)]
pub fn decode_batch(format: u8, input: &DeviceRows, in_len: u64, hashes: &DeviceBuffer, padding: u32,
                    out: &mut DeviceRows, status: &mut DeviceBuffer, scratch: &mut DeviceBuffer, stream: Stream)
                    -> Result<u64> {
    input.holds(input.count, in_len)?;
    if hashes.len() < input.count as usize * HASH_LEN || status.len() < input.count as usize * 4 ||
        (scratch.len() as u64) < decode_scratch_len(format, in_len, input.count) {
        return Err(ChipError::InvalidArgument);
    }
    let mut out_len = 0u64;
    check(unsafe {
        ffi::chip_decode_batch_dev(format, input.as_ptr(), input.stride, in_len, input.count, hashes.as_ptr(), padding,
                                   out.as_mut_ptr(), out.stride, &mut out_len, status.as_mut_ptr() as *mut u32,
                                   scratch.ptr, stream.0)
    })?;
    Ok(out_len)
}

/// scrub (decoding.rs:151-212) of every row: one result per stream
/// (Ok = repaired into that row of `out`; UnnecessaryScrub = intact).
/// Synchronous.
#[allow(clippy::too_many_arguments)]
pub fn scrub_batch(input: &DeviceRows, len: u64, hashes: &DeviceBuffer, padding: u32, chunk_len: u32,
                   out: &mut DeviceRows, scratch: &mut DeviceBuffer, stream: Stream) -> Result<Vec<Result<()>>> {
    input.holds(input.count, len)?;
    out.holds(input.count, len)?;
    if hashes.len() < input.count as usize * HASH_LEN ||
        (scratch.len() as u64) < unsafe { ffi::chip_scrub_scratch_len(len, input.count) } {
        return Err(ChipError::InvalidArgument);
    }
    let mut status = vec![0i32; input.count as usize];
    check(unsafe {
        ffi::chip_scrub_batch_dev(input.as_ptr(), input.stride, len, input.count, hashes.as_ptr(), padding, chunk_len,
                                  out.as_mut_ptr(), out.stride, status.as_mut_ptr(), scratch.ptr, stream.0)
    })?;
    Ok(status.into_iter().map(check).collect())
}

/// encode() of `count` objects in HOST memory, H2D / kernels / D2H and the
/// host stages overlapped over `nslots` device slots.  Returns the encoded
/// length of every object; streams at `out[o * out_stride..]`, hashes at
/// `hashes[32 o..]`.  At Zfec|Bao the library writes each stream's header and
/// data-shard chunks from the host and copies only the rest back; with a host
/// stage and `out` in pinned memory it also reads the device's input from
/// `out` (the call holds `&mut out` for its whole duration, so that is safe).
#[allow(clippy::too_many_arguments)]
pub fn encode_host_batch(format: u8, pubkey: &[u8], input: &[u8], n: usize, count: usize, in_stride: usize,
                         out: &mut [u8], out_stride: usize, hashes: &mut [u8], infos: Option<&mut [ChipEncodeInfo]>,
                         nslots: u32, slice_bytes: u64, host_threads: u32) -> Result<Vec<u64>> {
    let in_need = if count == 0 { 0 } else { (count - 1) * in_stride + n };
    if input.len() < in_need || out_stride < encode_max_len(n) || out.len() < count * out_stride ||
        hashes.len() < count * HASH_LEN ||
        infos.as_ref().map_or(false, |i| i.len() < count) {
        return Err(ChipError::InvalidArgument);
    }
    abi()?;
    let mut lens = vec![0u64; count];
    check(unsafe {
        ffi::chip_encode_host_batch(format, pubkey.as_ptr(), pubkey.len() as u64, ptr::null(), input.as_ptr(), n as u64,
                                    count as u64, in_stride as u64, out.as_mut_ptr(), out_stride as u64,
                                    lens.as_mut_ptr(), hashes.as_mut_ptr(),
                                    infos.map_or(ptr::null_mut(), |i| i.as_mut_ptr()), nslots, slice_bytes,
                                    host_threads)
    })?;
    Ok(lens)
}

/// decode() of `count` encodings in HOST memory; one result per object
/// (a corrupted object does not fail its neighbours).
#[allow(clippy::too_many_arguments)]
pub fn decode_host_batch(format: u8, secret_key: &[u8], hashes: &[u8], input: &[u8], in_len: &[u64],
                         in_stride: usize, padding: &[u32], out: &mut [u8], out_stride: usize, nslots: u32,
                         slice_bytes: u64, host_threads: u32) -> Result<Vec<Result<u64>>> {
    let count = in_len.len();
    if padding.len() < count || hashes.len() < count * HASH_LEN || out.len() < count * out_stride ||
        in_len.iter().enumerate().any(|(o, &l)| o * in_stride + l as usize > input.len()) {
        return Err(ChipError::InvalidArgument);
    }
    abi()?;
    let mut lens = vec![0u64; count];
    let mut status = vec![0i32; count];
    let rc = unsafe {
        ffi::chip_decode_host_batch(format, secret_key.as_ptr(), secret_key.len() as u64, hashes.as_ptr(),
                                    input.as_ptr(), in_len.as_ptr(), count as u64, in_stride as u64, padding.as_ptr(),
                                    out.as_mut_ptr(), out_stride as u64, lens.as_mut_ptr(), status.as_mut_ptr(),
                                    nslots, slice_bytes, host_threads)
    };
    if rc != ffi::CHIP_OK && status.iter().all(|&s| s == ffi::CHIP_OK) {
        return Err(ChipError::from_status(rc, 0, 0)); // a call-level failure, not an object's
    }
    Ok(status
        .into_iter()
        .zip(lens)
        .map(|(s, l)| if s == ffi::CHIP_OK { Ok(l) } else { Err(ChipError::from_status(s, HASH_LEN, l)) })
        .collect())
}

#[cfg(test)]
mod tests {
    use super::*;

    #[test]
    fn status_round_trip() {
        for s in [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 100, 101] {
            assert_eq!(ChipError::from_status(s, 31, 7).status(), s);
        }
    }

    #[test]
    fn size_helpers() {
        assert_eq!(calc_padding_len(16 << 20, 4).unwrap(), (0, 4 << 20));
        assert_eq!(bao_encoded_len(16 << 20), 35_651_528);
        assert_eq!(zfec_encoded_len(1243, 4, 8), 8192);
    }

    #[test]
    fn layouts_match_the_header() {
        assert_eq!(std::mem::size_of::<ChipEncodeInfo>(), 44);
        assert_eq!(std::mem::size_of::<ffi::chip_ecies_inject>(), 16);
        assert_eq!(std::mem::size_of::<ChipHeader>(), 152);
    }
}
