"""ctypes binding of libmaxio_ec.so (include/maxio_ec.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
maxio_amd/csrc``).  There is no fallback: if the shared object is missing or
fails to load, every entry point raises ``NativeLibraryMissing``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# MXEC_LIB: load another build of the library (A/B runs of a kernel change).
LIB_PATH = os.environ.get("MXEC_LIB") or os.path.join(_HERE, "lib", "libmaxio_ec.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "maxio_ec.h")

_lock = threading.Lock()
_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


class BodySums(ctypes.Structure):
    """mxec_body_sums: Md5 ETag + ChecksumHasher values (filesystem.rs:28-63)."""

    _fields_ = [
        ("md5", ctypes.c_uint8 * 16),
        ("crc32", ctypes.c_uint32),
        ("crc32c", ctypes.c_uint32),
        ("sha1", ctypes.c_uint8 * 20),
        ("sha256", ctypes.c_uint8 * 32),
    ]


class FramesJob(ctypes.Structure):
    """mxec_frames_job (encrypt-then-EC frames, storage/crypto.rs)."""

    _fields_ = [
        ("key", ctypes.c_void_p),
        ("nonce_prefix", ctypes.c_uint8 * 4),
        ("frame_size", ctypes.c_uint32),
        ("first_index", ctypes.c_uint64),
        ("aad_dev", ctypes.c_void_p),
        ("aad_len", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("in_dev", ctypes.c_void_p),
        ("len", ctypes.c_uint64),
        ("out_dev", ctypes.c_void_p),
    ]


class ChunkInfo(ctypes.Structure):
    """mxec_chunk_info == the reference's ChunkInfo (storage/mod.rs:182-189)."""

    _fields_ = [
        ("index", ctypes.c_uint32),
        ("size", ctypes.c_uint64),
        ("sha256", ctypes.c_char * 65),
        ("kind", ctypes.c_uint8),
    ]


class MultipartPart(ctypes.Structure):
    """mxec_multipart_part (PartMeta of a CompleteMultipartUpload)."""

    _fields_ = [
        ("path", ctypes.c_char_p),
        ("size", ctypes.c_uint64),
        ("md5", ctypes.c_uint8 * 16),
        ("part_number", ctypes.c_uint32),
        ("encrypted", ctypes.c_uint8),
    ]


class Object(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("m", ctypes.c_int32), ("shard_size", ctypes.c_uint64)]


P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
SZ = ctypes.c_size_t
U64 = ctypes.c_uint64
U64P = ctypes.POINTER(ctypes.c_uint64)
SZP = ctypes.POINTER(ctypes.c_size_t)
U8P = ctypes.POINTER(ctypes.c_uint8)
I32P = ctypes.POINTER(ctypes.c_int32)
INT = ctypes.c_int

_SIGS = {
    "mxec_version": (ctypes.c_char_p, []),
    "mxec_strerror": (ctypes.c_char_p, [INT]),
    "mxec_last_error": (ctypes.c_char_p, []),
    "mxec_device_count": (INT, []),
    "mxec_open": (P, [ctypes.c_uint32, INT]),
    "mxec_open_test": (P, [ctypes.c_uint32, INT, INT, ctypes.c_uint32, ctypes.c_uint64]),
    "mxec_close": (None, [P]),
    "mxec_ctx_device_count": (INT, [P]),
    "mxec_ctx_device_id": (INT, [P, INT]),
    "mxec_ctx_combiner_stats": (INT, [P, INT, U64P, U64P]),
    "mxec_ctx_pipe_stats": (INT, [P, INT, U64P, INT]),
    "mxec_ctx_rs_grid": (INT, [P, INT, INT, INT, U64]),
    "mxec_ctx_coef_stats": (INT, [P, INT, U64P, U64P, U64P]),
    "mxec_host_alloc": (P, [P, ctypes.c_size_t]),
    "mxec_host_alloc_device": (P, [P, INT, ctypes.c_size_t]),
    "mxec_batch_alloc": (P, [P, INT, INT, INT, U64, U64, U64P, ctypes.POINTER(ctypes.c_float)]),
    "mxec_batch_free": (INT, [P, P]),
    "mxec_host_free": (None, [P, P]),
    "mxec_rs_check": (INT, [INT, INT]),
    "mxec_rs_parity_matrix": (INT, [INT, INT, U8P]),
    "mxec_sha256_batch": (INT, [P, PP, SZP, SZ, U8P]),
    "mxec_encode": (INT, [P, INT, INT, SZ, PP, SZP, PP, U8P]),
    "mxec_reconstruct": (INT, [P, INT, INT, SZ, PP, SZP, U8P, U8P, ctypes.c_uint32, ctypes.POINTER(INT)]),
    "mxec_encode_strided_device": (
        INT, [P, INT, P, INT, INT, U64, U64, P, U64, U64, U64P, P, U64, U64, P]),
    "mxec_encode_batch_device": (INT, [P, INT, P, ctypes.POINTER(Object), U64, PP, U64P, PP, P]),
    "mxec_encode_batch_host": (INT, [P, ctypes.POINTER(Object), U64, PP, U64P, PP, U8P, I32P]),
    "mxec_reconstruct_batch_host": (INT, [P, ctypes.POINTER(Object), U64, PP, U64P, U8P, U8P, ctypes.c_uint32, I32P]),
    "mxec_reconstruct_strided_device": (
        INT, [P, INT, P, INT, INT, U64, U64, P, U64, U64, U64P, U8P, P, ctypes.c_uint32, I32P]),
    "mxec_reconstruct_batch_device": (
        INT, [P, INT, P, ctypes.POINTER(Object), U64, PP, U64P, U8P, P, ctypes.c_uint32, I32P]),
    "mxec_reconstruct_batch_device_async": (
        INT, [P, INT, P, ctypes.POINTER(Object), U64, PP, U64P, U8P, P, ctypes.c_uint32, I32P,
              ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_sha256_batch_device": (INT, [P, INT, P, PP, U64P, U64, P]),
    "mxec_write_chunk": (INT, [P, ctypes.c_char_p, ctypes.c_uint32, P, SZ, ctypes.POINTER(ChunkInfo)]),
    "mxec_compute_and_write_parity": (
        INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, ctypes.POINTER(ChunkInfo), INT, ctypes.POINTER(ChunkInfo)]),
    "mxec_put_object_chunked": (INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, P, SZ]),
    "mxec_put_object_chunked_sums": (INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, P, SZ,
                                           ctypes.c_uint32, P]),
    "mxec_body_sums_batch": (INT, [P, PP, U64P, U64, ctypes.c_uint32, P]),
    "mxec_put_object_chunked_encrypted": (INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, P, P, P,
                                                ctypes.c_uint32, P, SZ, ctypes.c_uint32, P]),
    "mxec_complete_multipart_chunked": (INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32,
                                              ctypes.POINTER(MultipartPart), ctypes.c_uint32, ctypes.c_char_p]),
    "mxec_complete_multipart_chunked_encrypted": (
        INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, ctypes.POINTER(MultipartPart), ctypes.c_uint32, P,
              ctypes.c_char_p, P, P, P, ctypes.c_uint32, ctypes.c_char_p]),
    "mxec_frames_len": (U64, [U64, ctypes.c_uint32]),
    "mxec_frames_encrypt": (INT, [P, P, P, U64, P, ctypes.c_uint32, ctypes.c_uint32, P, U64, P, U64, U64P]),
    "mxec_frames_decrypt": (INT, [P, P, U64, P, ctypes.c_uint32, ctypes.c_uint32, P, U64, U64, P, U64, U64P]),
    "mxec_frames_encrypt_device": (INT, [P, INT, P, P, U64]),
    "mxec_frames_decrypt_device": (INT, [P, INT, P, P, U64, ctypes.POINTER(ctypes.c_int32)]),
    "mxec_frame_aads": (INT, [P, P, ctypes.c_uint32, U64, U64, P]),
    "mxec_body_sums_batch_device": (INT, [P, INT, P, PP, U64P, U64, ctypes.c_uint32, P]),
    "mxec_get_object_chunked": (INT, [P, ctypes.c_char_p, U64, U64, P, U64, U64P]),
    "mxec_get_object_chunked_encrypted": (INT, [P, ctypes.c_char_p, P, P, ctypes.c_uint32, ctypes.c_uint32, U64,
                                                U64, U64, P, U64, U64P]),
    "mxec_try_reconstruct_data_chunk": (INT, [P, ctypes.c_char_p, ctypes.c_uint32, P, U64, U64P]),
    "mxec_reader_open": (INT, [P, ctypes.c_char_p, U64, U64, U64, ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_reader_read": (ctypes.c_int64, [P, P, U64]),
    "mxec_reader_close": (None, [P]),
    "mxec_ticket_fd": (INT, [P]),
    "mxec_ticket_poll": (INT, [P]),
    "mxec_ticket_wait": (INT, [P]),
    "mxec_ticket_error": (ctypes.c_char_p, [P]),
    "mxec_ticket_free": (None, [P]),
    "mxec_sha256_batch_async": (INT, [P, PP, SZP, SZ, U8P, ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_encode_async": (INT, [P, INT, INT, SZ, PP, SZP, PP, U8P, ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_reconstruct_async": (INT, [P, INT, INT, SZ, PP, SZP, U8P, U8P, ctypes.c_uint32, ctypes.POINTER(INT),
                                     ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_put_object_chunked_async": (INT, [P, ctypes.c_char_p, U64, ctypes.c_uint32, P, SZ,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_get_object_chunked_async": (INT, [P, ctypes.c_char_p, U64, U64, P, U64, U64P,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "mxec_reconstruct_strided_device_async": (
        INT, [P, INT, P, INT, INT, U64, U64, P, U64, U64, U64P, U8P, P, ctypes.c_uint32, I32P,
              ctypes.POINTER(ctypes.c_void_p)]),
}


def lib() -> ctypes.CDLL:
    """Load libmaxio_ec.so once; raise loudly if it is not there."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not built: run __graft_entry__.build() or make -C maxio_amd/csrc")
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment specific
            raise NativeLibraryMissing(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def declared_symbols() -> list[str]:
    """Every function declared in include/maxio_ec.h."""
    import re

    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(mxec_[a-z0-9_]+)\s*\(", text)))
