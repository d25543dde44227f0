"""maxio_amd — MI355X erasure-coding backend for MaxIO's chunked-EC path.

Reed–Solomon GF(2^8) encode / reconstruct and per-chunk SHA-256 run as HIP
kernels for gfx950 inside libmaxio_ec.so; include/maxio_ec.h is the C ABI a
Rust ``extern "C"`` block binds.  This package is the
Python mirror of that ABI used by the tests and bench.py.
"""
from .ec import (  # noqa: F401
    DATA_ONLY,
    SUM_CRC32,
    SUM_CRC32C,
    SUM_MD5,
    SUM_SHA1,
    SUM_SHA256,
    ChunkReader,
    put_result,
    Context,
    ReedSolomon,
    RSError,
    Ticket,
    device_count,
    parity_matrix,
    rs_check,
    version,
)
from ._native import LIB_PATH, NativeLibraryMissing, declared_symbols, lib  # noqa: F401

__all__ = [
    "Context",
    "ReedSolomon",
    "RSError",
    "DATA_ONLY",
    "SUM_MD5",
    "SUM_CRC32",
    "SUM_CRC32C",
    "SUM_SHA1",
    "SUM_SHA256",
    "ChunkReader",
    "put_result",
    "device_count",
    "parity_matrix",
    "version",
    "rs_check",
    "lib",
    "LIB_PATH",
    "NativeLibraryMissing",
    "declared_symbols",
]
