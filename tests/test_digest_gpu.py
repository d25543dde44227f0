"""GPU: PUT body digests (mxec_body_sums_batch*, digest_kernel.hip) against
the oracle (oracle/body_oracle.c, pinned by tests/test_oracle_body.py),
hashlib and zlib — bit-exact.  Lengths straddle every boundary the kernels
have: 64-byte blocks (55/56/64 tails), 16-byte CRC units, 4 KiB CRC rows and
128 KiB CRC tiles; device pointers at every 16-byte misalignment."""
from __future__ import annotations

import hashlib
import zlib

import numpy as np
import pytest

import maxio_amd
import oracle

pytestmark = pytest.mark.gpu

ALL = 0x1F
TILE = 128 << 10
LENGTHS = [0, 1, 15, 16, 17, 55, 56, 63, 64, 65, 119, 120, 128, 4095, 4096, 4097,
           TILE - 1, TILE, TILE + 1, 3 * TILE + 4096 + 5, (1 << 20) + 13]


def _body(n: int, seed: int = 0) -> bytes:
    return np.random.default_rng(1000 + n + seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _check(d: dict, body: bytes):
    assert d["md5"] == hashlib.md5(body).digest()
    assert d["sha1"] == hashlib.sha1(body).digest()
    assert d["sha256"] == hashlib.sha256(body).digest()
    assert d["crc32"] == zlib.crc32(body)
    assert d["crc32c"] == oracle.crc32c(body)


def test_body_sums_lengths_one_batch(ctx):
    bodies = [_body(n) for n in LENGTHS]
    for d, b in zip(ctx.body_sums(bodies, ALL), bodies):
        _check(d, b)


@pytest.mark.parametrize("which", [maxio_amd.SUM_MD5, maxio_amd.SUM_CRC32C,
                                   maxio_amd.SUM_CRC32 | maxio_amd.SUM_SHA1])
def test_body_sums_subsets(ctx, which):
    body = _body(300_001, 3)
    d = ctx.body_sums([body], which)[0]
    assert set(d) == {k for k, f in [("md5", 1), ("crc32", 2), ("crc32c", 4), ("sha1", 8), ("sha256", 16)]
                      if which & f}
    if "md5" in d:
        assert d["md5"] == hashlib.md5(body).digest()
    if "crc32c" in d:
        assert d["crc32c"] == oracle.crc32c(body)
    if "crc32" in d:
        assert d["crc32"] == zlib.crc32(body)
    if "sha1" in d:
        assert d["sha1"] == hashlib.sha1(body).digest()


def test_body_sums_device_unaligned(ctx):
    """Device pointers at every offset mod 16, lengths crossing rows/tiles."""
    import torch

    src = _body(4 * TILE + 4096, 7)
    buf = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    base = buf.data_ptr()
    cases = [(off, ln) for off in range(16) for ln in (0, 5, 16, 100, 4096 + 3, TILE + 17)]
    cases += [(1, 3 * TILE + 4000), (15, 4 * TILE - 16)]
    out = torch.zeros(len(cases) * 76, dtype=torch.uint8, device="cuda")
    ctx.body_sums_device([base + o for o, _ in cases], [n for _, n in cases], out.data_ptr(), ALL)
    torch.cuda.synchronize()
    rec = out.cpu().numpy().reshape(len(cases), 76)
    for (o, n), r in zip(cases, rec):
        body = src[o:o + n]
        assert r[0:16].tobytes() == hashlib.md5(body).digest(), (o, n)
        assert int.from_bytes(r[16:20].tobytes(), "little") == zlib.crc32(body), (o, n)
        assert int.from_bytes(r[20:24].tobytes(), "little") == oracle.crc32c(body), (o, n)
        assert r[24:44].tobytes() == hashlib.sha1(body).digest(), (o, n)
        assert r[44:76].tobytes() == hashlib.sha256(body).digest(), (o, n)


def test_crc_large_body_and_many_bodies(ctx):
    """A 96 MiB body (768 tiles over several workgroups) and 300 small ones."""
    big = _body(96 << 20, 11)
    small = [_body(int(n), 12) for n in np.random.default_rng(5).integers(0, 20000, 300)]
    res = ctx.body_sums([big] + small, maxio_amd.SUM_CRC32 | maxio_amd.SUM_CRC32C)
    assert res[0]["crc32"] == zlib.crc32(big)
    assert res[0]["crc32c"] == oracle.crc32c(big)
    for d, b in zip(res[1:], small):
        assert d["crc32"] == zlib.crc32(b) and d["crc32c"] == oracle.crc32c(b)


def test_put_result_matches_reference_tests(ctx, tmp_path):
    """integration.rs:2943-2962 (CRC32 of b"hello checksum world") and
    :3029-3052 (CRC32C of b"compute my checksum please"), base64 of the
    big-endian value; ETag = quoted hex MD5 (filesystem.rs:775-776)."""
    import base64

    body = b"hello checksum world"
    r = ctx.put_object_chunked_sums(str(tmp_path / "a.ec"), 8, 2, body, "CRC32")
    assert r["checksum_value"] == base64.b64encode(zlib.crc32(body).to_bytes(4, "big")).decode()
    assert r["etag"] == '"%s"' % hashlib.md5(body).hexdigest()
    assert ctx.get_object_chunked(str(tmp_path / "a.ec")) == body
    body = b"compute my checksum please"
    r = ctx.put_object_chunked_sums(str(tmp_path / "b.ec"), 10, 0, body, "CRC32C")
    assert r["checksum_value"] == oracle.put_checksum_b64("CRC32C", body)
    for algo in ("SHA1", "SHA256"):
        r = ctx.put_object_chunked_sums(str(tmp_path / f"{algo}.ec"), 1 << 20, 2, body, algo)
        assert r["checksum_value"] == oracle.put_checksum_b64(algo, body)
    r = ctx.put_object_chunked_sums(str(tmp_path / "e.ec"), 100, 2, b"")
    assert r == {"etag": '"d41d8cd98f00b204e9800998ecf8427e"'}
