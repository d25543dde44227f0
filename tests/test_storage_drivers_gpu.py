"""GPU: the other chunking drivers of SURVEY §8(a8) — put_object_chunked_encrypted
(filesystem.rs:835-1060), complete_multipart_chunked (:1147-1310) and
complete_multipart_chunked_encrypted (:1315-1560) — through the C ABI, checked
file by file and byte for byte against the layout the reference writes
(oracle frames / parity, hashlib digests, to_string_pretty manifest), the
ETags, and a GET + frame-decrypt round trip."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

import maxio_amd
import oracle
from helpers import expected_ec_object

pytestmark = pytest.mark.gpu

FS = oracle.FRAME_CHUNK_SIZE


def _rand(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _check_dir(ec: str, files: dict, manifest: str):
    assert sorted(os.listdir(ec)) == sorted(list(files) + ["manifest.json"])
    assert open(os.path.join(ec, "manifest.json")).read() == manifest
    for name, want in files.items():
        assert open(os.path.join(ec, name), "rb").read() == want, name


def _object_aads(prefix: bytes, n: int):
    return [oracle.frame_aad(prefix, i) for i in range(n)]


@pytest.mark.parametrize("n,chunk,m", [(0, 100000, 2), (1000, 100000, 2), (3 * FS + 17, 100000, 2),
                                       (2 * FS, 2 * (FS + 28), 3), (FS + 5, 1 << 20, 0)])
def test_put_object_chunked_encrypted_layout(ctx, tmp_path, n, chunk, m):
    key, prefix = _rand(32, n + 1), bytes([9, 8, 7, 6])
    idp = oracle.object_aad_prefix("bkt", "dir/obj.bin", None)
    body = _rand(n, n)
    ec = str(tmp_path / "obj.ec")
    res = ctx.put_object_chunked_encrypted(ec, chunk, m, key, prefix, idp, body, checksum_algo="CRC32C")
    nfr = (n + FS - 1) // FS
    ct = oracle.frames_encrypt(key, prefix, body, _object_aads(idp, nfr) or None)
    files, man = expected_ec_object(ct, chunk, m, plaintext_size=n)
    _check_dir(ec, files, man)
    assert res["etag"] == '"' + hashlib.md5(body).hexdigest() + '"'
    assert res["checksum_value"] == oracle.put_checksum_b64("CRC32C", body)
    # GET the frame stream back (degraded when there is parity) and decrypt it
    if m and n:
        os.unlink(os.path.join(ec, "000000"))
    got = ctx.get_object_chunked(ec)
    assert got == ct
    assert ctx.frames_decrypt(key, got, n, _object_aads(idp, nfr) or None) == body


def _write_parts(tmp_path, sizes, seed):
    parts, bodies = [], []
    for i, sz in enumerate(sizes):
        b = _rand(sz, seed + i)
        p = tmp_path / f"part{i + 1}"
        p.write_bytes(b)
        parts.append({"path": str(p), "size": sz, "etag": hashlib.md5(b).hexdigest(), "part_number": i + 1})
        bodies.append(b)
    return parts, bodies


@pytest.mark.parametrize("sizes,chunk,m", [([5 << 20, 5 << 20, 123457], 1 << 20, 2), ([0], 4096, 2),
                                           ([70000, 1], 65536, 4), ([300, 200], 1000, 0)])
def test_complete_multipart_chunked_layout_and_etag(ctx, tmp_path, sizes, chunk, m):
    parts, bodies = _write_parts(tmp_path, sizes, 50)
    ec = str(tmp_path / "mp.ec")
    etag = ctx.complete_multipart_chunked(ec, chunk, m, parts)
    whole = b"".join(bodies)
    files, man = expected_ec_object(whole, chunk, m)
    _check_dir(ec, files, man)
    raw = b"".join(bytes.fromhex(p["etag"]) for p in parts)
    assert etag == f'"{hashlib.md5(raw).hexdigest()}-{len(parts)}"'
    assert ctx.get_object_chunked(ec) == whole


def test_complete_multipart_chunked_encrypted(ctx, tmp_path):
    """SSE multipart: part 1 stored encrypted under the upload key (part AADs),
    part 2 plain; the object is re-encrypted under a fresh key."""
    upload_key, upload_id = _rand(32, 1), "upl-7f3a"
    key, prefix = _rand(32, 2), b"NPFX"
    idp = oracle.object_aad_prefix("b", "k", None)
    p1, p2 = _rand(3 * FS + 1000, 3), _rand(40000, 4)
    part_prefix = b"PART\0" + upload_id.encode() + b"\0" + (1).to_bytes(4, "little") + b"\0"
    n1 = (len(p1) + FS - 1) // FS
    enc1 = oracle.frames_encrypt(upload_key, b"UPLD", p1, _object_aads(part_prefix, n1))
    (tmp_path / "part1").write_bytes(enc1)
    (tmp_path / "part2").write_bytes(p2)
    parts = [{"path": str(tmp_path / "part1"), "size": len(p1), "etag": hashlib.md5(p1).hexdigest(),
              "part_number": 1, "encrypted": True},
             {"path": str(tmp_path / "part2"), "size": len(p2), "etag": hashlib.md5(p2).hexdigest(),
              "part_number": 2}]
    ec = str(tmp_path / "mpe.ec")
    etag = ctx.complete_multipart_chunked_encrypted(ec, 1 << 20, 2, parts, upload_key, upload_id, key, prefix, idp)
    plain = p1 + p2
    nfr = (len(plain) + FS - 1) // FS
    ct = oracle.frames_encrypt(key, prefix, plain, _object_aads(idp, nfr))
    files, man = expected_ec_object(ct, 1 << 20, 2, plaintext_size=len(plain))
    _check_dir(ec, files, man)
    raw = bytes.fromhex(parts[0]["etag"]) + bytes.fromhex(parts[1]["etag"])
    assert etag == f'"{hashlib.md5(raw).hexdigest()}-2"'
    # a tampered encrypted part fails the completion with the decryptor's error
    bad = bytearray(enc1)
    bad[100] ^= 1
    (tmp_path / "part1").write_bytes(bytes(bad))
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.complete_multipart_chunked_encrypted(str(tmp_path / "x.ec"), 1 << 20, 2, parts, upload_key,
                                                 upload_id, key, prefix, idp)
    assert "authentication" in str(e.value)


def test_get_object_chunked_encrypted_ranges(ctx, tmp_path):
    """GET and ranged GET of an encrypt-then-EC object: frames covering the
    range read through the verified reader (degraded here: a data shard is
    gone), decrypted, sliced — equal to the plaintext slice."""
    key, prefix = _rand(32, 11), b"RNGE"
    idp = oracle.object_aad_prefix("bkt", "ranged", "v7")
    n = 5 * FS + 4321
    body = _rand(n, 12)
    ec = str(tmp_path / "r.ec")
    ctx.put_object_chunked_encrypted(ec, 100003, 3, key, prefix, idp, body)
    os.unlink(os.path.join(ec, "000001"))
    assert ctx.get_object_chunked_encrypted(ec, key, idp) == body
    rng = np.random.default_rng(5)
    cases = [(0, 1), (FS - 1, 2), (FS, FS), (n - 1, 1), (3 * FS + 7, None), (0, n), (n - 10, 100)]
    cases += [(int(o), int(ln)) for o, ln in zip(rng.integers(0, n, 8), rng.integers(1, 3 * FS, 8))]
    for off, ln in cases:
        want = body[off:] if ln is None else body[off:off + ln]
        assert ctx.get_object_chunked_encrypted(ec, key, idp, off, ln) == want, (off, ln)
    # the wrong identity (another key's AAD) fails authentication
    with pytest.raises(maxio_amd.RSError):
        ctx.get_object_chunked_encrypted(ec, key, oracle.object_aad_prefix("bkt", "other", "v7"))


def test_multipart_errors(ctx, tmp_path):
    """A missing part file is an IO error; an encrypted part without the
    upload key is refused; the plain driver refuses encrypted parts."""
    parts, _ = _write_parts(tmp_path, [1000, 2000], 90)
    parts.append({"path": str(tmp_path / "nope"), "size": 5, "etag": "00" * 16, "part_number": 3})
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.complete_multipart_chunked(str(tmp_path / "a.ec"), 4096, 2, parts)
    assert e.value.code == -40 and e.value.name == "Io"
    enc = [dict(parts[0], encrypted=True)]
    with pytest.raises(maxio_amd.RSError):
        ctx.complete_multipart_chunked(str(tmp_path / "b.ec"), 4096, 2, enc)
