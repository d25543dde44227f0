"""GPU: the reference's EC integration scenarios (tests/integration.rs
:2702-2898, :3155-3385, :5646-5700) replayed at the file level through the
C ABI's write / parity / verify / reconstruct functions.  Fault injection is
done the way the reference tests do it: by editing chunk files."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

import maxio_amd
from helpers import scenario_body

pytestmark = pytest.mark.gpu


def _put(ctx, tmp_path, golden, name):
    sc = golden("reference_scenarios.json")[name]
    body = scenario_body(sc["body"])
    ec = str(tmp_path / f"{name}.bin.ec")
    ctx.put_object_chunked(ec, sc["chunk_size"], sc["parity_shards"], body)
    return sc, body, ec


@pytest.mark.parametrize("name", [
    "parity_write_0xAB_350", "parity_read_0xCD_350", "v1_no_parity_0xAA_2048", "empty_with_parity",
    "ec_put_get_0x42_3072", "ec_plus_parity_k49", "parity_range_per_chunk_350",
])
def test_layout_and_manifest_bytes(ctx, tmp_path, golden, name):
    sc, body, ec = _put(ctx, tmp_path, golden, name)
    files = sorted(os.listdir(ec))
    assert files == sorted(list(sc["files"]) + ["manifest.json"])
    assert open(os.path.join(ec, "manifest.json")).read() == sc["manifest"]
    for fname, meta in sc["files"].items():
        raw = open(os.path.join(ec, fname), "rb").read()
        assert len(raw) == meta["size"]
        if "hex" in meta:
            assert raw.hex() == meta["hex"], fname
    # digest format pinned by integration.rs:5699-5700: hex(sha256(raw chunk))
    man = json.loads(sc["manifest"])
    for c in man["chunks"]:
        raw = open(os.path.join(ec, f"{c['index']:06}"), "rb").read()
        assert c["sha256"] == hashlib.sha256(raw).hexdigest()
    assert ctx.get_object_chunked(ec) == body


def test_parity_write_structure(ctx, tmp_path, golden):
    """integration.rs:3155 — 4 data + 2 parity + manifest = 7 entries, v2."""
    _, _, ec = _put(ctx, tmp_path, golden, "parity_write_0xAB_350")
    assert len(os.listdir(ec)) == 7
    man = json.load(open(os.path.join(ec, "manifest.json")))
    assert man["version"] == 2 and man["chunk_count"] == 4 and man["parity_shards"] == 2
    assert len(man["chunks"]) == 6
    assert all("kind" not in man["chunks"][i] for i in range(4))
    assert man["chunks"][4]["kind"] == "parity" and man["chunks"][5]["kind"] == "parity"


def test_recovery_corrupted_chunk(ctx, tmp_path, golden):
    """integration.rs:3214 — chunk 1 overwritten with 100 zero bytes."""
    _, body, ec = _put(ctx, tmp_path, golden, "parity_corrupt_0xEF_350")
    open(os.path.join(ec, "000001"), "wb").write(bytes(100))
    assert ctx.get_object_chunked(ec) == body
    assert ctx.try_reconstruct_data_chunk(ec, 1) == body[100:200]


def test_recovery_missing_chunk(ctx, tmp_path, golden):
    """integration.rs:3239 — chunk 0 deleted."""
    _, body, ec = _put(ctx, tmp_path, golden, "parity_missing_0x42_350")
    os.remove(os.path.join(ec, "000000"))
    assert ctx.get_object_chunked(ec) == body


def test_too_many_failures(ctx, tmp_path, golden):
    """integration.rs:3263 — 3 chunks deleted with m=2: must fail."""
    _, _, ec = _put(ctx, tmp_path, golden, "parity_too_many_0x77_350")
    for i in range(3):
        os.remove(os.path.join(ec, f"{i:06}"))
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.get_object_chunked(ec)
    assert e.value.name == "TooFewShardsPresent"
    assert "only 3 of 4 required shards available" in str(e.value)


def test_range_read_degraded(ctx, tmp_path, golden):
    """integration.rs:3299 — per-chunk bytes, chunk 1 corrupted, bytes=50-149."""
    _, body, ec = _put(ctx, tmp_path, golden, "parity_range_per_chunk_350")
    open(os.path.join(ec, "000001"), "wb").write(bytes(100))
    assert ctx.get_object_chunked(ec, 50, 100) == body[50:150]
    assert ctx.get_object_chunked(ec, 340, 10) == body[340:350]


def test_empty_object_is_v1(ctx, tmp_path, golden):
    """integration.rs:3357 — empty object: version 1, no parity fields."""
    _, _, ec = _put(ctx, tmp_path, golden, "empty_with_parity")
    man = json.load(open(os.path.join(ec, "manifest.json")))
    assert man["version"] == 1 and "parity_shards" not in man
    assert ctx.get_object_chunked(ec) == b""


def test_bitrot_without_parity_is_an_error(ctx, tmp_path, golden):
    """integration.rs:2860 — no parity + corrupt chunk: never the original bytes."""
    _, _, ec = _put(ctx, tmp_path, golden, "ec_put_get_0x42_3072")
    raw = bytearray(open(os.path.join(ec, "000001"), "rb").read())
    raw[10] ^= 0xFF
    open(os.path.join(ec, "000001"), "wb").write(raw)
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.get_object_chunked(ec)
    assert e.value.name == "Integrity" and "checksum mismatch on chunk 1" in str(e.value)


def test_ec_plus_parity_k49_recovery(ctx, tmp_path, golden):
    """integration.rs:5646 shape — 50 000 B at 1 KiB chunks, m=2 (k=49)."""
    _, body, ec = _put(ctx, tmp_path, golden, "ec_plus_parity_k49")
    open(os.path.join(ec, "000001"), "wb").write(bytes(1024))
    os.remove(os.path.join(ec, "000048"))
    assert ctx.get_object_chunked(ec) == body


def test_write_chunk_then_parity_path(ctx, tmp_path, golden):
    """write_chunk per chunk + compute_and_write_parity (re-reads the files,
    filesystem.rs:1108-1113) produce the same files as the batched path."""
    sc = golden("reference_scenarios.json")["parity_range_per_chunk_350"]
    body = scenario_body(sc["body"])
    ec = tmp_path / "x.ec"
    ec.mkdir()
    infos = [ctx.write_chunk(str(ec), j, body[j * 100:(j + 1) * 100]) for j in range(4)]
    pinfos = ctx.compute_and_write_parity(str(ec), 100, 2, infos)
    man = json.loads(sc["manifest"])
    assert infos + pinfos == man["chunks"]
    for fname, meta in sc["files"].items():
        if "hex" in meta:
            assert (ec / fname).read_bytes().hex() == meta["hex"]


def test_parity_guard_255(ctx, tmp_path):
    ec = tmp_path / "big.ec"
    with pytest.raises(maxio_amd.RSError) as e:
        ctx.put_object_chunked(str(ec), 4, 10, bytes(4 * 250))
    assert e.value.name == "TooManyShards255"
    assert "Increase --chunk-size" in str(e.value)


def test_baseline_config1_loopback(ctx, tmp_path):
    """BASELINE configs[0]: one 10 MiB object with --chunk-size 10485760
    --parity-shards 2 (k=1: parity rows are [1], both parity files are copies
    of the data), delete one shard file (000000), GET still returns the body."""
    import numpy as np

    body = np.random.default_rng(1).integers(0, 256, 10 << 20, dtype=np.uint8).tobytes()
    ec = tmp_path / "obj.bin.ec"
    ctx.put_object_chunked(str(ec), 10 << 20, 2, body)
    assert sorted(os.listdir(ec)) == ["000000", "000001", "000002", "manifest.json"]
    assert (ec / "000001").read_bytes() == body and (ec / "000002").read_bytes() == body
    man = json.loads((ec / "manifest.json").read_text())
    assert man["chunks"][0]["sha256"] == hashlib.sha256(body).hexdigest()
    os.remove(ec / "000000")
    assert ctx.get_object_chunked(str(ec)) == body


def test_several_bad_chunks_one_decode(ctx, tmp_path):
    """Two bad chunks in one range (m=2): both rebuilt, byte-exact."""
    import numpy as np

    body = np.random.default_rng(2).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    ec = tmp_path / "x.ec"
    ctx.put_object_chunked(str(ec), 128, 2, body)          # k = 8
    open(ec / "000002", "wb").write(bytes(128))             # corrupt
    os.remove(ec / "000006")                                # missing
    assert ctx.get_object_chunked(str(ec)) == body
    assert ctx.get_object_chunked(str(ec), 200, 700) == body[200:900]
    os.remove(ec / "000009")                                # a parity shard too: 3 erasures > m
    with pytest.raises(maxio_amd.RSError):
        ctx.get_object_chunked(str(ec))


def _drain(reader, step):
    out = bytearray()
    while True:
        b = reader.read(step)
        if not b:
            return bytes(out)
        assert len(b) <= step
        out += b


@pytest.mark.parametrize("batch_bytes", [0, 1, 300])
@pytest.mark.parametrize("step", [1, 7, 100, 4096])
def test_reader_streams_ranges(ctx, tmp_path, batch_bytes, step):
    """VerifiedChunkReader (chunk_reader.rs:35-226): any read size, any batch
    size, ranges that start and end mid-chunk, one chunk rebuilt."""
    import numpy as np

    body = np.random.default_rng(3).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    ec = tmp_path / "r.ec"
    ctx.put_object_chunked(str(ec), 128, 2, body)
    open(ec / "000003", "wb").write(bytes(5))
    for off, ln in [(0, None), (0, 1000), (130, 1), (127, 2), (200, 700), (999, 1), (1000, 5), (500, 10**6)]:
        with ctx.open_reader(str(ec), off, ln, batch_bytes) as r:
            want = body[off:] if ln is None else body[off:off + ln]
            assert _drain(r, step) == want, (off, ln)


def test_reader_serves_healthy_prefix_then_fails(ctx, tmp_path):
    """Without parity a corrupt chunk fails the stream only when it is reached
    (chunk_reader.rs:87-152): every byte before it has been delivered."""
    import numpy as np

    body = np.random.default_rng(4).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    ec = tmp_path / "np.ec"
    ctx.put_object_chunked(str(ec), 128, 0, body)
    raw = bytearray((ec / "000003").read_bytes())
    raw[0] ^= 1
    (ec / "000003").write_bytes(raw)
    for batch_bytes in (0, 128):
        with ctx.open_reader(str(ec), 0, None, batch_bytes) as r:
            got = bytearray()
            with pytest.raises(maxio_amd.RSError) as e:
                while True:
                    b = r.read(50)
                    if not b:
                        break
                    got += b
            assert bytes(got) == body[:3 * 128]
            assert e.value.name == "Integrity" and "checksum mismatch on chunk 3" in str(e.value)
    # a range that ends before the bad chunk never touches it
    with ctx.open_reader(str(ec), 10, 300) as r:
        assert _drain(r, 64) == body[10:310]


def _get_raw(ctx, ec, off, ln, cap):
    """mxec_get_object_chunked as called from C: (rc, bytes written)."""
    import ctypes

    import numpy as np

    out = np.full(max(cap, 1), 0xEE, np.uint8)
    n = ctypes.c_uint64(0)
    rc = maxio_amd.lib().mxec_get_object_chunked(ctx.handle, str(ec).encode(), off,
                                                  (1 << 64) - 1 if ln is None else ln,
                                                  out.ctypes.data, cap, ctypes.byref(n))
    return rc, out[: n.value].tobytes()


def _drain_raw(ctx, ec, off, ln):
    """The streaming reader over the same range: (rc, bytes before the error)."""
    got = bytearray()
    try:
        with ctx.open_reader(str(ec), off, ln, 1 << 40) as r:
            while True:
                b = r.read(333)
                if not b:
                    return 0, bytes(got)
                got += b
    except maxio_amd.RSError as e:
        return e.code, bytes(got)


@pytest.mark.parametrize("window", [None, "1", "300"])
@pytest.mark.parametrize("damage", ["none", "missing", "corrupt", "short", "missing+corrupt",
                                    "missing+parity", "too_many", "no_parity_corrupt"])
def test_one_shot_get_matches_streaming_reader(ctx_with, tmp_path, damage, window):
    """The one-shot GET reads whole chunks straight into the caller's buffer
    and, with a chunk known bad before hashing, verifies and rebuilds in one
    mxec_reconstruct call; the streaming reader goes chunk buffer by chunk
    buffer.  Same bytes, same length, same error, over ranges that start and
    end mid-chunk, for every kind of damage, with the one-shot GET's chunk
    window at its default, one chunk (window 1) and two chunks (300)."""
    import numpy as np

    ctx = ctx_with(MXEC_GET_WINDOW=window)  # read at mxec_open; None: the default

    body = np.random.default_rng(9).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    ec = tmp_path / "o.ec"
    ctx.put_object_chunked(str(ec), 128, 0 if damage == "no_parity_corrupt" else 3, body)  # k = 8

    def corrupt(i):
        raw = bytearray((ec / f"{i:06}").read_bytes())
        raw[5] ^= 0x40
        (ec / f"{i:06}").write_bytes(raw)

    if damage == "missing":
        os.remove(ec / "000002")
    elif damage == "corrupt":
        corrupt(4)
    elif damage == "short":
        (ec / "000001").write_bytes(bytes(7))
    elif damage == "missing+corrupt":
        os.remove(ec / "000002")
        corrupt(6)
    elif damage == "missing+parity":
        os.remove(ec / "000000")
        corrupt(9)
        os.remove(ec / "000010")
    elif damage == "too_many":
        os.remove(ec / "000002")
        corrupt(3)
        corrupt(5)
        os.remove(ec / "000008")
    elif damage == "no_parity_corrupt":
        corrupt(3)
    for off, ln in [(0, None), (0, 1000), (130, 1), (127, 2), (200, 700), (256, 384), (999, 1), (5, 995)]:
        want_len = len(body[off:] if ln is None else body[off:off + ln])
        rc, got = _get_raw(ctx, ec, off, ln, want_len)
        rrc, rgot = _drain_raw(ctx, ec, off, ln)
        assert (rc, got) == (rrc, rgot), (damage, off, ln, rc, rrc, len(got), len(rgot))
        if rc == 0:
            assert got == (body[off:] if ln is None else body[off:off + ln])
    if damage in ("none", "missing", "corrupt", "short", "missing+corrupt", "missing+parity"):
        assert ctx.get_object_chunked(str(ec)) == body


@pytest.mark.parametrize("edit,code", [
    (lambda j: j.replace('"version": 2,', ""), -42),                      # missing required field
    (lambda j: j.replace('"kind": "parity"', '"kind": "Parity"', 1), -42),  # unknown variant
    (lambda j: j.replace('"chunk_count": 3', '"chunk_count": 4294967299'), -42),  # u32 overflow
    (lambda j: j.replace('"chunk_size": 4096', '"chunk_size": 4096.0'), -42),     # float for u64
    (lambda j: j + " x", -42),                                            # trailing characters
    (lambda j: j.replace('"total_size"', '"extra": ' + "[" * 200 + "]" * 200 + ', "total_size"'), -42),
    (lambda j: j.replace('"version": 2', '"versio\\u006e": 2'), 0),       # escaped key is the same key
    (lambda j: j.replace('"version": 2,', '"version": 2, "future_field": {"a": [1, 2.5]},'), 0),
])
def test_get_manifest_parsed_like_serde(ctx, tmp_path, edit, code):
    """GET reads manifest.json with the serde-exact reader (manifest.cpp):
    what serde_json::from_str::<ChunkManifest> rejects is MXEC_E_JSON
    (StorageError::Json, filesystem.rs:3171), what it accepts reads back."""
    body = np.random.default_rng(51).integers(0, 256, 3 * 4096 - 5, dtype=np.uint8)
    ec = tmp_path / "m.ec"
    ctx.put_object_chunked(str(ec), 4096, 2, body)
    mpath = ec / "manifest.json"
    text = mpath.read_text()
    assert '"chunk_count": 3' in text and '"version": 2' in text
    mpath.write_text(edit(text))
    if code == 0:
        assert ctx.get_object_chunked(str(ec)) == body.tobytes()
    else:
        with pytest.raises(maxio_amd.RSError) as ei:
            ctx.get_object_chunked(str(ec), capacity=body.size)
        assert ei.value.code == code, str(ei.value)
        assert "JSON error" in str(ei.value)


def test_get_manifest_not_utf8_is_io_error(ctx, tmp_path):
    body = np.random.default_rng(52).integers(0, 256, 5000, dtype=np.uint8)
    ec = tmp_path / "u.ec"
    ctx.put_object_chunked(str(ec), 4096, 1, body)
    mpath = ec / "manifest.json"
    raw = mpath.read_bytes().replace(b'"version"', b'"v\xffersion"')
    mpath.write_bytes(raw)
    with pytest.raises(maxio_amd.RSError) as ei:
        ctx.get_object_chunked(str(ec), capacity=body.size)
    assert ei.value.code == -40
