//! maxio-ec-sys — raw FFI to libmaxio_ec.so, the MI355X erasure-coding
//! backend for MaxIO's chunked-EC storage path (`include/maxio_ec.h`).
//!
//! Every item here mirrors the C header one for one: same names, same
//! argument order, same integer widths (`int` = `c_int`, `size_t` = `usize`,
//! `uint64_t` = `u64`), `const` pointees as `*const`.  The repository's CPU
//! test `tests/test_rust_ffi.py` parses this file and the header and fails
//! when either side drifts (symbols, arity, argument widths, struct layouts,
//! constants).  No Rust toolchain exists in the build image, so this crate is
//! kept consistent mechanically rather than compiled there; INTEGRATION.md
//! shows the call sites in MaxIO it replaces (filesystem.rs:1062 write_chunk,
//! :1084 compute_and_write_parity, chunk_reader.rs:157
//! try_reconstruct_data_chunk, chunk_reader.rs:87 load_chunk_sync).
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

/// `mxec_ctx`: one per process, shared by every tokio worker (all entry
/// points are thread-safe).
#[repr(C)]
pub struct MxecCtx {
    _p: [u8; 0],
}

/// `mxec_reader`: VerifiedChunkReader as a pull stream.
#[repr(C)]
pub struct MxecReader {
    _p: [u8; 0],
}

/// `mxec_ticket`: completion handle of an `*_async` call.
#[repr(C)]
pub struct MxecTicket {
    _p: [u8; 0],
}

/// `mxec_object`: (k, m, shard_size) of one object of a batch.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct MxecObject {
    pub k: i32,
    pub m: i32,
    pub shard_size: u64,
}

/// `mxec_chunk_info` == ChunkInfo (storage/mod.rs:182-189); kind 0 = data, 1 = parity.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct MxecChunkInfo {
    pub index: u32,
    pub size: u64,
    pub sha256: [c_char; 65],
    pub kind: u8,
}

/// `mxec_body_sums`: Md5 ETag + ChecksumHasher values (filesystem.rs:28-63).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct MxecBodySums {
    pub md5: [u8; 16],
    pub crc32: u32,
    pub crc32c: u32,
    pub sha1: [u8; 20],
    pub sha256: [u8; 32],
}

/// `mxec_frames_job`: one body of a device-resident encrypt-then-EC batch.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct MxecFramesJob {
    pub key: *const u8,
    pub nonce_prefix: [u8; 4],
    pub frame_size: u32,
    pub first_index: u64,
    pub aad_dev: *const u8,
    pub aad_len: u32,
    pub reserved: u32,
    pub in_dev: *const u8,
    pub len: u64,
    pub out_dev: *mut u8,
}

/// `mxec_multipart_part`: one part of CompleteMultipartUpload (PartMeta).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct MxecMultipartPart {
    pub path: *const c_char,
    pub size: u64,
    pub md5: [u8; 16],
    pub part_number: u32,
    pub encrypted: u8,
}

// ---- mxec_ctx_pipe_stats counter indices ----------------------------------
pub const MXEC_PIPE_STAT_COPIES_1D: c_int = 0;
pub const MXEC_PIPE_STAT_COPIES_2D: c_int = 1;
pub const MXEC_PIPE_STAT_ROWS_2D: c_int = 2;
pub const MXEC_PIPE_STAT_WAVE_BLOCKS: c_int = 3;
pub const MXEC_PIPE_STAT_SDMA_CHECKS: c_int = 4;
pub const MXEC_PIPE_STAT_SDMA_SLOW: c_int = 5;
pub const MXEC_PIPE_STAT_VERIFY_WAVES: c_int = 6;
pub const MXEC_PIPE_STAT_VERIFY_GROUPS: c_int = 7;
pub const MXEC_PIPE_STAT_SDMA_LAST_MBPS: c_int = 8;
pub const MXEC_PIPE_STAT_SDMA_DOWN_CHECKS: c_int = 9;
pub const MXEC_PIPE_STAT_SDMA_DOWN_SLOW: c_int = 10;
pub const MXEC_PIPE_STAT_SDMA_DOWN_LAST_MBPS: c_int = 11;
pub const MXEC_PIPE_STAT_CALLS: c_int = 12;
pub const MXEC_PIPE_STAT_CALLS_SHARED: c_int = 13;
pub const MXEC_PIPE_STAT_SPEC_PIECES: c_int = 14;
pub const MXEC_PIPE_STAT_SPEC_REDOS: c_int = 15;
pub const MXEC_PIPE_STAT_PACE_WAITS: c_int = 16;
pub const MXEC_PIPE_STAT_COUNT: c_int = 17;

// ---- return codes (reed_solomon_erasure::Error one for one, then MaxIO's) --
pub const MXEC_OK: c_int = 0;
pub const MXEC_E_TOO_FEW_SHARDS: c_int = -1;
pub const MXEC_E_TOO_MANY_SHARDS: c_int = -2;
pub const MXEC_E_TOO_FEW_DATA_SHARDS: c_int = -3;
pub const MXEC_E_TOO_MANY_DATA_SHARDS: c_int = -4;
pub const MXEC_E_TOO_FEW_PARITY_SHARDS: c_int = -5;
pub const MXEC_E_TOO_MANY_PARITY_SHARDS: c_int = -6;
pub const MXEC_E_TOO_FEW_BUFFER_SHARDS: c_int = -7;
pub const MXEC_E_TOO_MANY_BUFFER_SHARDS: c_int = -8;
pub const MXEC_E_INCORRECT_SHARD_SIZE: c_int = -9;
pub const MXEC_E_TOO_FEW_SHARDS_PRESENT: c_int = -10;
pub const MXEC_E_EMPTY_SHARD: c_int = -11;
pub const MXEC_E_INVALID_SHARD_FLAGS: c_int = -12;
pub const MXEC_E_INVALID_INDEX: c_int = -13;
pub const MXEC_E_SINGULAR_MATRIX: c_int = -14;
pub const MXEC_E_TOO_MANY_SHARDS_255: c_int = -20;
pub const MXEC_E_INVALID_ARG: c_int = -21;
pub const MXEC_E_DEVICE: c_int = -30;
pub const MXEC_E_OOM: c_int = -31;
pub const MXEC_E_NO_DEVICE: c_int = -32;
pub const MXEC_E_IO: c_int = -40;
pub const MXEC_E_INTEGRITY: c_int = -41;
pub const MXEC_E_JSON: c_int = -42;

pub const MXEC_F_DATA_ONLY: u32 = 0x1;
pub const MXEC_FRAME_CHUNK_SIZE: u32 = 65536;
pub const MXEC_FRAME_OVERHEAD: u32 = 28;
pub const MXEC_SUM_MD5: u32 = 0x01;
pub const MXEC_SUM_CRC32: u32 = 0x02;
pub const MXEC_SUM_CRC32C: u32 = 0x04;
pub const MXEC_SUM_SHA1: u32 = 0x08;
pub const MXEC_SUM_SHA256: u32 = 0x10;

extern "C" {
    pub fn mxec_version() -> *const c_char;
    pub fn mxec_strerror(code: c_int) -> *const c_char;
    pub fn mxec_last_error() -> *const c_char;
    pub fn mxec_device_count() -> c_int;
    pub fn mxec_open(device_mask: u32, streams_per_device: c_int) -> *mut MxecCtx;
    /// Test-only open (tests drive the multi-device and grid-stride paths with it).
    pub fn mxec_open_test(device_mask: u32, streams_per_device: c_int, logical_devices: c_int, rs_grid_cap: u32,
                          coef_arena_bytes: u64) -> *mut MxecCtx;
    pub fn mxec_close(ctx: *mut MxecCtx);
    pub fn mxec_ctx_device_count(ctx: *const MxecCtx) -> c_int;
    pub fn mxec_ctx_device_id(ctx: *const MxecCtx, i: c_int) -> c_int;
    pub fn mxec_ctx_combiner_stats(ctx: *mut MxecCtx, i: c_int, launches: *mut u64, messages: *mut u64) -> c_int;
    pub fn mxec_ctx_pipe_stats(ctx: *mut MxecCtx, dev: c_int, out: *mut u64, n: c_int) -> c_int;
    pub fn mxec_ctx_rs_grid(ctx: *mut MxecCtx, dev: c_int, k: c_int, m: c_int, shard_size: u64) -> c_int;
    pub fn mxec_ctx_coef_stats(ctx: *mut MxecCtx, dev: c_int, recycles: *mut u64, relaunches: *mut u64,
                               fence_waits: *mut u64) -> c_int;
    pub fn mxec_host_alloc(ctx: *mut MxecCtx, bytes: usize) -> *mut c_void;
    pub fn mxec_host_alloc_device(ctx: *mut MxecCtx, dev: c_int, bytes: usize) -> *mut c_void;
    pub fn mxec_batch_alloc(ctx: *mut MxecCtx, dev: c_int, k: c_int, m: c_int, shard_size: u64, n_obj: u64,
                            shard_stride: *mut u64, probe_ms: *mut f32) -> *mut c_void;
    pub fn mxec_batch_free(ctx: *mut MxecCtx, p: *mut c_void) -> c_int;
    pub fn mxec_host_free(ctx: *mut MxecCtx, p: *mut c_void);
    pub fn mxec_rs_check(k: c_int, m: c_int) -> c_int;
    pub fn mxec_rs_parity_matrix(k: c_int, m: c_int, out: *mut u8) -> c_int;
    pub fn mxec_sha256_batch(ctx: *mut MxecCtx, bufs: *const *const u8, lens: *const usize, n: usize, out: *mut [u8; 32]) -> c_int;
    pub fn mxec_encode(ctx: *mut MxecCtx, k: c_int, m: c_int, shard_size: usize, data: *const *const u8, data_len: *const usize, parity: *const *mut u8, sha256_out: *mut [u8; 32]) -> c_int;
    pub fn mxec_reconstruct(ctx: *mut MxecCtx, k: c_int, m: c_int, shard_size: usize, shards: *const *mut u8, shard_len: *const usize, expected_sha256: *const [u8; 32], present_inout: *mut u8, flags: u32, n_present: *mut c_int) -> c_int;
    pub fn mxec_ticket_fd(t: *const MxecTicket) -> c_int;
    pub fn mxec_ticket_poll(t: *mut MxecTicket) -> c_int;
    pub fn mxec_ticket_wait(t: *mut MxecTicket) -> c_int;
    pub fn mxec_ticket_error(t: *const MxecTicket) -> *const c_char;
    pub fn mxec_ticket_free(t: *mut MxecTicket);
    pub fn mxec_sha256_batch_async(ctx: *mut MxecCtx, bufs: *const *const u8, lens: *const usize, n: usize, out: *mut [u8; 32], ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_encode_async(ctx: *mut MxecCtx, k: c_int, m: c_int, shard_size: usize, data: *const *const u8, data_len: *const usize, parity: *const *mut u8, sha256_out: *mut [u8; 32], ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_reconstruct_async(ctx: *mut MxecCtx, k: c_int, m: c_int, shard_size: usize, shards: *const *mut u8, shard_len: *const usize, expected_sha256: *const [u8; 32], present_inout: *mut u8, flags: u32, n_present: *mut c_int, ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_put_object_chunked_async(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, body: *const u8, len: usize, ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_get_object_chunked_async(ctx: *mut MxecCtx, ec_dir: *const c_char, offset: u64, length: u64, out: *mut u8, out_cap: u64, out_len: *mut u64, ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_encode_strided_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, k: c_int, m: c_int, shard_size: u64, n_obj: u64, data: *const u8, data_obj_stride: u64, data_shard_stride: u64, data_len: *const u64, parity: *mut u8, parity_obj_stride: u64, parity_shard_stride: u64, digests_dev: *mut u8) -> c_int;
    pub fn mxec_encode_batch_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, objs: *const MxecObject, n_obj: u64, data: *const *const u8, data_len: *const u64, parity: *const *mut u8, digests_dev: *mut u8) -> c_int;
    pub fn mxec_encode_batch_host(ctx: *mut MxecCtx, objs: *const MxecObject, n_obj: u64, data: *const *const u8, data_len: *const u64, parity: *const *mut u8, digests: *mut [u8; 32], status_out: *mut i32) -> c_int;
    pub fn mxec_reconstruct_batch_host(ctx: *mut MxecCtx, objs: *const MxecObject, n_obj: u64, shards: *const *mut u8, shard_len: *const u64, present: *mut u8, expected_sha256: *const [u8; 32], flags: u32, status_out: *mut i32) -> c_int;
    pub fn mxec_reconstruct_strided_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, k: c_int, m: c_int, shard_size: u64, n_obj: u64, shards: *mut u8, obj_stride: u64, shard_stride: u64, shard_len: *const u64, present: *mut u8, expected_sha_dev: *const u8, flags: u32, status_out: *mut i32) -> c_int;
    pub fn mxec_reconstruct_batch_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, objs: *const MxecObject, n_obj: u64, shards: *const *mut u8, shard_len: *const u64, present: *mut u8, expected_sha_dev: *const u8, flags: u32, status_out: *mut i32) -> c_int;
    pub fn mxec_reconstruct_batch_device_async(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, objs: *const MxecObject, n_obj: u64, shards: *const *mut u8, shard_len: *const u64, present: *mut u8, expected_sha_dev: *const u8, flags: u32, status_out: *mut i32, ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_reconstruct_strided_device_async(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, k: c_int, m: c_int, shard_size: u64, n_obj: u64, shards: *mut u8, obj_stride: u64, shard_stride: u64, shard_len: *const u64, present: *mut u8, expected_sha_dev: *const u8, flags: u32, status_out: *mut i32, ticket: *mut *mut MxecTicket) -> c_int;
    pub fn mxec_sha256_batch_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, bufs: *const *const u8, lens: *const u64, n: u64, digests_dev: *mut u8) -> c_int;
    pub fn mxec_write_chunk(ctx: *mut MxecCtx, ec_dir: *const c_char, index: u32, data: *const u8, len: usize, out: *mut MxecChunkInfo) -> c_int;
    pub fn mxec_compute_and_write_parity(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, data_chunks: *const MxecChunkInfo, k: c_int, parity_out: *mut MxecChunkInfo) -> c_int;
    pub fn mxec_put_object_chunked(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, body: *const u8, len: usize) -> c_int;
    pub fn mxec_frames_len(plaintext_len: u64, frame_size: u32) -> u64;
    pub fn mxec_frames_encrypt(ctx: *mut MxecCtx, key: *const u8, nonce_prefix: *const u8, first_index: u64, aad: *const u8, aad_len: u32, frame_size: u32, pt: *const u8, len: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn mxec_frames_decrypt(ctx: *mut MxecCtx, key: *const u8, first_index: u64, aad: *const u8, aad_len: u32, frame_size: u32, frames: *const u8, frames_len: u64, plaintext_size: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn mxec_frames_encrypt_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, jobs: *const MxecFramesJob, n_jobs: u64) -> c_int;
    pub fn mxec_frames_decrypt_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, jobs: *const MxecFramesJob, n_jobs: u64, status_out: *mut i32) -> c_int;
    pub fn mxec_frame_aads(ctx: *mut MxecCtx, prefix: *const u8, prefix_len: u32, first_index: u64, n_frames: u64, out: *mut [u8; 32]) -> c_int;
    pub fn mxec_body_sums_batch(ctx: *mut MxecCtx, bodies: *const *const u8, lens: *const u64, n: u64, which: u32, out: *mut MxecBodySums) -> c_int;
    pub fn mxec_body_sums_batch_device(ctx: *mut MxecCtx, dev: c_int, stream: *mut c_void, bodies_dev: *const *const u8, lens: *const u64, n: u64, which: u32, out_dev: *mut MxecBodySums) -> c_int;
    pub fn mxec_put_object_chunked_sums(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, body: *const u8, len: usize, which: u32, sums_out: *mut MxecBodySums) -> c_int;
    pub fn mxec_put_object_chunked_encrypted(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, key: *const u8, nonce_prefix: *const u8, aad_prefix: *const u8, aad_prefix_len: u32, body: *const u8, len: usize, which: u32, sums_out: *mut MxecBodySums) -> c_int;
    pub fn mxec_complete_multipart_chunked(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, parts: *const MxecMultipartPart, n_parts: u32, etag_out: *mut c_char) -> c_int;
    pub fn mxec_complete_multipart_chunked_encrypted(ctx: *mut MxecCtx, ec_dir: *const c_char, chunk_size: u64, parity_shards: u32, parts: *const MxecMultipartPart, n_parts: u32, upload_key: *const u8, upload_id: *const c_char, key: *const u8, nonce_prefix: *const u8, aad_prefix: *const u8, aad_prefix_len: u32, etag_out: *mut c_char) -> c_int;
    pub fn mxec_get_object_chunked(ctx: *mut MxecCtx, ec_dir: *const c_char, offset: u64, length: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn mxec_get_object_chunked_encrypted(ctx: *mut MxecCtx, ec_dir: *const c_char, key: *const u8, aad_prefix: *const u8, aad_prefix_len: u32, frame_size: u32, plaintext_size: u64, offset: u64, length: u64, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
    pub fn mxec_reader_open(ctx: *mut MxecCtx, ec_dir: *const c_char, offset: u64, length: u64, batch_bytes: u64, out: *mut *mut MxecReader) -> c_int;
    pub fn mxec_reader_read(r: *mut MxecReader, buf: *mut u8, cap: u64) -> i64;
    pub fn mxec_reader_close(r: *mut MxecReader);
    pub fn mxec_try_reconstruct_data_chunk(ctx: *mut MxecCtx, ec_dir: *const c_char, target: u32, out: *mut u8, out_cap: u64, out_len: *mut u64) -> c_int;
}

/// The calling thread's last error message (`mxec_last_error`).
pub fn last_error() -> String {
    unsafe { std::ffi::CStr::from_ptr(mxec_last_error()).to_string_lossy().into_owned() }
}
