"""CPU: pin the PUT body-digest oracle (oracle/body_oracle.c) — MD5 (ETag),
CRC32, CRC32C, SHA-1, SHA-256 as filesystem.rs:28-63 / :700-777 compute them —
against hashlib / zlib, the published check values and the reference's own
checksum tests.  No GPU."""
from __future__ import annotations

import base64
import hashlib
import zlib

import numpy as np
import pytest

import oracle

LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4096, 65536 + 7]


def _data(n: int, seed: int = 0) -> bytes:
    return np.random.default_rng(seed + n).integers(0, 256, n, dtype=np.uint8).tobytes()


def _py_crc32c(data: bytes, crc: int = 0) -> int:
    """Independent table-driven CRC32C (Castagnoli, reflected 0x82F63B78)."""
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        table.append(c)
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c = (c >> 8) ^ table[(c ^ b) & 0xFF]
    return c ^ 0xFFFFFFFF


@pytest.mark.parametrize("n", LENGTHS)
def test_md5_sha1_crc32_match_hashlib_zlib(n):
    d = _data(n)
    assert oracle.md5(d) == hashlib.md5(d).digest()
    assert oracle.sha1(d) == hashlib.sha1(d).digest()
    assert oracle.crc32(d) == zlib.crc32(d)


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 1000])
def test_crc32c_matches_independent_restatement(n):
    d = _data(n, 5)
    assert oracle.crc32c(d) == _py_crc32c(d)


def test_check_values():
    # Standard "123456789" check values of both CRCs, RFC 1321 / FIPS vectors.
    assert oracle.crc32(b"123456789") == 0xCBF43926
    assert oracle.crc32c(b"123456789") == 0xE3069283
    assert oracle.md5(b"").hex() == "d41d8cd98f00b204e9800998ecf8427e"
    assert oracle.md5(b"abc").hex() == "900150983cd24fb0d6963f7d28e17f72"
    assert oracle.sha1(b"abc").hex() == "a9993e364706816aba3e25717850c26c9cd0d89d"


def test_crc32c_rfc3720_vectors():
    # RFC 3720 B.4 (iSCSI CRC32C examples), as the u32 value.
    assert oracle.crc32c(bytes(32)) == 0x8A9136AA
    assert oracle.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert oracle.crc32c(bytes(range(32))) == 0x46DD794E
    assert oracle.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 1000, 65537])
def test_crc32c_fast_form_matches(n):
    d = _data(n, 13)
    assert oracle.crc32c(d, fast=True) == oracle.crc32c(d)
    assert oracle.crc32c(d, 0x12345678, fast=True) == oracle.crc32c(d, 0x12345678)


def test_crc32c_append_is_streaming():
    # crc32c_append(v, b) continues crc32c(a): ChecksumHasher::update (:45-52).
    d = _data(5000, 9)
    for cut in (0, 1, 7, 64, 4999, 5000):
        assert oracle.crc32c(d[cut:], oracle.crc32c(d[:cut])) == oracle.crc32c(d)


def test_reference_checksum_tests():
    # integration.rs:2943-2945: crc32fast::hash(b"hello checksum world"),
    # base64 of to_be_bytes; :3050 crc32c::crc32c(b"compute my checksum please").
    body = b"hello checksum world"
    want = base64.b64encode(zlib.crc32(body).to_bytes(4, "big")).decode()
    assert oracle.put_checksum_b64("CRC32", body) == want
    body = b"compute my checksum please"
    want = base64.b64encode(_py_crc32c(body).to_bytes(4, "big")).decode()
    assert oracle.put_checksum_b64("CRC32C", body) == want
    assert oracle.put_checksum_b64("SHA1", body) == base64.b64encode(hashlib.sha1(body).digest()).decode()
    assert oracle.put_checksum_b64("SHA256", body) == base64.b64encode(hashlib.sha256(body).digest()).decode()
