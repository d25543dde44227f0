"""ctypes wrapper of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU baseline.  The
product (maxio_amd/) never imports, links or calls anything under oracle/.
See oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_gf_mul.restype = ctypes.c_uint8
        L.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_div.restype = ctypes.c_uint8
        L.orc_gf_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_exp.restype = ctypes.c_uint8
        L.orc_gf_exp.argtypes = [ctypes.c_uint8, ctypes.c_size_t]
        L.orc_rs_check.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_rs_matrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.orc_rs_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_rs_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.orc_sha256.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_sha256_fast.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.orc_crc32.restype = ctypes.c_uint32
        L.orc_crc32c_append.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.orc_crc32c_append.restype = ctypes.c_uint32
        L.orc_crc32c_append_fast.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.orc_crc32c_append_fast.restype = ctypes.c_uint32
        L.orc_aes256_expand.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_aes256_encrypt_block.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_gf128_mul.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_gcm_encrypt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_gcm_decrypt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_frames_encrypt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]
        L.orc_frames_decrypt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_md5.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_sha1.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_compute_parity_ex.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int]
        L.orc_have_sha_ni.argtypes = []
        L.orc_try_reconstruct_data_chunk_ex.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def _arr(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b.reshape(-1).view(np.uint8))
    return np.frombuffer(bytes(b), np.uint8)


def _pp(arrs) -> ctypes.Array:
    return (ctypes.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])


def gf_mul(a: int, b: int) -> int:
    return int(lib().orc_gf_mul(a, b))


def gf_div(a: int, b: int) -> int:
    return int(lib().orc_gf_div(a, b))


def gf_exp(a: int, n: int) -> int:
    return int(lib().orc_gf_exp(a, n))


def rs_check(k: int, m: int) -> int:
    return int(lib().orc_rs_check(k, m))


def matrix(k: int, m: int) -> np.ndarray:
    out = np.zeros((k + m, k), np.uint8)
    rc = lib().orc_rs_matrix(k, m, out.ctypes.data)
    if rc:
        raise ValueError(rc)
    return out


def encode(data: Sequence, m: int, size: Optional[int] = None) -> list[np.ndarray]:
    """ReedSolomon::new(k, m).encode over k equal-size (or zero-padded to
    `size`) data shards; returns the m parity shards."""
    k = len(data)
    arrs = [_arr(d) for d in data]
    size = size if size is not None else arrs[0].size
    shards = [np.zeros(size, np.uint8) for _ in range(k + m)]
    for j, a in enumerate(arrs):
        shards[j][: a.size] = a
    rc = lib().orc_rs_encode(k, m, size, _pp(shards))
    if rc:
        raise ValueError(rc)
    return shards[k:]


def reconstruct(shards: Sequence[Optional[object]], k: int, m: int, size: int,
                data_only: bool = False) -> tuple[list[np.ndarray], np.ndarray, int]:
    bufs, present = [], np.zeros(k + m, np.uint8)
    for i in range(k + m):
        b = np.zeros(size, np.uint8)
        if shards[i] is not None:
            a = _arr(shards[i])
            b[: a.size] = a
            present[i] = 1
        bufs.append(b)
    rc = lib().orc_rs_reconstruct(k, m, size, _pp(bufs), present.ctypes.data, int(data_only))
    return bufs, present, int(rc)


def sha256(data, fast: bool = False) -> bytes:
    a = _arr(data)
    out = np.zeros(32, np.uint8)
    ptr = a.ctypes.data if a.size else np.zeros(1, np.uint8).ctypes.data
    (lib().orc_sha256_fast if fast else lib().orc_sha256)(ptr, a.size, out.ctypes.data)
    return out.tobytes()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else np.zeros(1, np.uint8).ctypes.data


def crc32(data) -> int:
    """crc32fast::hash (filesystem.rs:28-63 CRC32 arm)."""
    a = _arr(data)
    return int(lib().orc_crc32(_ptr(a), a.size))


def crc32c(data, crc: int = 0, fast: bool = False) -> int:
    """crc32c::crc32c_append(crc, data) (CRC32C arm); fast = SSE4.2 form."""
    a = _arr(data)
    f = lib().orc_crc32c_append_fast if fast else lib().orc_crc32c_append
    return int(f(crc, _ptr(a), a.size))


def md5(data) -> bytes:
    a = _arr(data)
    out = np.zeros(16, np.uint8)
    lib().orc_md5(_ptr(a), a.size, out.ctypes.data)
    return out.tobytes()


def sha1(data) -> bytes:
    a = _arr(data)
    out = np.zeros(20, np.uint8)
    lib().orc_sha1(_ptr(a), a.size, out.ctypes.data)
    return out.tobytes()


FRAME_CHUNK_SIZE = 65536  # crypto.rs:46


def aes256_block(key: bytes, block: bytes) -> bytes:
    rk = np.zeros(240, np.uint8)
    k = _arr(key)
    lib().orc_aes256_expand(k.ctypes.data, rk.ctypes.data)
    b = _arr(block)
    out = np.zeros(16, np.uint8)
    lib().orc_aes256_encrypt_block(rk.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out.tobytes()


def gf128_mul(x: bytes, y: bytes) -> bytes:
    a, b = _arr(x), _arr(y)
    out = np.zeros(16, np.uint8)
    lib().orc_gf128_mul(a.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out.tobytes()


def gcm_encrypt(key: bytes, iv: bytes, pt, aad=b"") -> tuple[bytes, bytes]:
    k, v, p, a = _arr(key), _arr(iv), _arr(pt), _arr(aad)
    ct = np.zeros(max(1, p.size), np.uint8)
    tag = np.zeros(16, np.uint8)
    lib().orc_gcm_encrypt(k.ctypes.data, v.ctypes.data, _ptr(a), a.size, _ptr(p), p.size, ct.ctypes.data,
                          tag.ctypes.data)
    return ct[:p.size].tobytes(), tag.tobytes()


def gcm_decrypt(key: bytes, iv: bytes, ct, tag: bytes, aad=b"") -> Optional[bytes]:
    k, v, c, a, t = _arr(key), _arr(iv), _arr(ct), _arr(aad), _arr(tag)
    pt = np.zeros(max(1, c.size), np.uint8)
    rc = lib().orc_gcm_decrypt(k.ctypes.data, v.ctypes.data, _ptr(a), a.size, _ptr(c), c.size, t.ctypes.data,
                               pt.ctypes.data)
    return None if rc else pt[:c.size].tobytes()


def frames_len(n: int, frame_size: int = FRAME_CHUNK_SIZE) -> int:
    return n + 28 * ((n + frame_size - 1) // frame_size)


def frames_encrypt(key: bytes, prefix: bytes, pt, aads: Optional[Sequence[bytes]] = None,
                   first_index: int = 0, frame_size: int = FRAME_CHUNK_SIZE) -> bytes:
    """FrameEncryptor over a whole buffer; aads[i] = AAD of frame i (equal lengths)."""
    p = _arr(pt)
    out = np.zeros(max(1, frames_len(p.size, frame_size)), np.uint8)
    a = _arr(b"".join(aads)) if aads else np.zeros(0, np.uint8)
    alen = len(aads[0]) if aads else 0
    lib().orc_frames_encrypt(_arr(key).ctypes.data, _arr(prefix).ctypes.data, first_index,
                             a.ctypes.data if aads else None, alen, frame_size, _ptr(p), p.size, out.ctypes.data)
    return out[:frames_len(p.size, frame_size)].tobytes()


def frames_decrypt(key: bytes, frames, plaintext_size: int, aads: Optional[Sequence[bytes]] = None,
                   first_index: int = 0, frame_size: int = FRAME_CHUNK_SIZE):
    """FrameDecryptor over a whole buffer -> (rc, plaintext)."""
    f = _arr(frames)
    out = np.zeros(max(1, plaintext_size), np.uint8)
    a = _arr(b"".join(aads)) if aads else np.zeros(0, np.uint8)
    alen = len(aads[0]) if aads else 0
    rc = lib().orc_frames_decrypt(_arr(key).ctypes.data, first_index, a.ctypes.data if aads else None, alen,
                                  frame_size, _ptr(f), plaintext_size, out.ctypes.data)
    return int(rc), out[:plaintext_size].tobytes()


def frame_aad(prefix: bytes, index: int) -> bytes:
    """build_frame_aad / build_part_aad (filesystem.rs:118-158): SHA-256 of the
    identity prefix || chunk_index as u64 LE."""
    import hashlib

    return hashlib.sha256(prefix + index.to_bytes(8, "little")).digest()


def object_aad_prefix(bucket: str, key: str, version_id: Optional[str] = None) -> bytes:
    return bucket.encode() + b"\0" + key.encode() + b"\0" + (version_id or "").encode() + b"\0"


def put_checksum_b64(algo: str, data) -> str:
    """ChecksumHasher::finalize_base64 (filesystem.rs:55-63)."""
    import base64

    if algo == "CRC32":
        raw = crc32(data).to_bytes(4, "big")
    elif algo == "CRC32C":
        raw = crc32c(data).to_bytes(4, "big")
    elif algo == "SHA1":
        raw = sha1(data)
    elif algo == "SHA256":
        raw = sha256(data)
    else:
        raise ValueError(algo)
    return base64.b64encode(raw).decode()


def have_sha_ni() -> bool:
    """Whether this host has the x86 SHA extensions (sha2 0.10.9's backend)."""
    return bool(lib().orc_have_sha_ni())


def compute_parity(data: Sequence, m: int, chunk_size: int, sha_ni: bool = False):
    """filesystem.rs:1084-1145 minus I/O: (parity shards, k+m digests, rc).
    sha_ni: digests by the SHA-NI form (the timed CPU baseline; sha2 0.10.9
    auto-selects it on x86-64), else the scalar restatement (the checker)."""
    arrs = [_arr(d) for d in data]
    k = len(arrs)
    parity = [np.zeros(chunk_size, np.uint8) for _ in range(max(m, 0))]
    lens = (ctypes.c_size_t * max(1, k))(*[a.size for a in arrs])
    dig = np.zeros((k + max(m, 0)) * 32 or 32, np.uint8)
    src = [a if a.size else np.zeros(1, np.uint8) for a in arrs]
    rc = lib().orc_compute_parity_ex(k, m, chunk_size, _pp(src), lens, _pp(parity), dig.ctypes.data, int(sha_ni))
    digests = [dig[32 * i: 32 * i + 32].tobytes() for i in range(k + max(m, 0))]
    return parity, digests, int(rc)


def try_reconstruct_data_chunk(shards: Sequence[Optional[object]], k: int, m: int,
                               shard_size: int, expected: Sequence[bytes],
                               chunk_sizes: Sequence[int], target: int, sha_ni: bool = False):
    """chunk_reader.rs:157-226 minus I/O: (bytes or None, rc, n_present).
    sha_ni as compute_parity."""
    total = k + m
    arrs = [None if s is None else _arr(s) for s in shards]
    keep = [a if (a is not None and a.size) else np.zeros(1, np.uint8) for a in arrs]
    ptrs = (ctypes.c_void_p * total)(*[None if arrs[i] is None else keep[i].ctypes.data
                                       for i in range(total)])
    lens = (ctypes.c_size_t * total)(*[0 if a is None else a.size for a in arrs])
    exp = np.frombuffer(b"".join(expected), np.uint8).copy()
    sizes = (ctypes.c_uint64 * total)(*chunk_sizes)
    out = np.zeros(max(1, shard_size), np.uint8)
    npres = ctypes.c_int(0)
    rc = lib().orc_try_reconstruct_data_chunk_ex(k, m, shard_size, ptrs, lens, exp.ctypes.data,
                                                 sizes, target, out.ctypes.data, ctypes.byref(npres), int(sha_ni))
    if rc:
        return None, int(rc), npres.value
    return out[: chunk_sizes[target]].tobytes(), 0, npres.value
