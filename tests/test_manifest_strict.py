"""CPU: the ChunkManifest reader of libmaxio_ec.so (maxio_amd/csrc/manifest.cpp)
accepts exactly what serde_json::from_str::<ChunkManifest> accepts
(storage/mod.rs:164-189, read at filesystem.rs:3171), built on its own with
-fsanitize=address,undefined together with the C oracle (oracle/*.c), and
fed one malformed manifest per rule.  Every rejection is what serde reports
as StorageError::Json (MXEC_E_JSON in the library); bytes that are not
UTF-8 fail earlier, in read_to_string, as an I/O error.

Expected outcomes restate serde / serde_json 1.0 behaviour for this struct
(no deny_unknown_fields; `kind` rename_all = "lowercase" with a default;
Option fields with #[serde(default)]); parity with serde itself is unpinned
(no Rust toolchain here), the cases follow its documented rules."""
from __future__ import annotations

import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.join(ROOT, "tests", "c_manifest")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")

SHA = "ab" * 32
CHUNK = '{"index": 0, "size": 10, "sha256": "%s"}' % SHA


def base(**over) -> str:
    """A valid manifest with fields overridden (value strings are raw JSON;
    None drops the field)."""
    fields = {"version": "2", "total_size": "10", "chunk_size": "10", "chunk_count": "1",
              "chunks": "[" + CHUNK + ', {"index": 1, "size": 10, "sha256": "%s", "kind": "parity"}]' % SHA,
              "parity_shards": "1", "shard_size": "10"}
    fields.update(over)
    return "{" + ", ".join(f'"{k}": {v}' for k, v in fields.items() if v is not None) + "}"


def chunk(**over) -> str:
    f = {"index": "0", "size": "10", "sha256": f'"{SHA}"'}
    f.update(over)
    inner = "{" + ", ".join(f'"{k}": {v}' for k, v in f.items() if v is not None) + "}"
    return base(chunks="[" + inner + "]", parity_shards=None, shard_size=None, version="1")


# (name, text, expected error substring or None for accepted)
CASES = [
    ("valid_v2", base(), None),
    ("valid_writer_format", '{\n  "version": 1,\n  "total_size": 0,\n  "chunk_size": 4096,\n  "chunk_count": 1,\n'
     '  "chunks": [\n    {\n      "index": 0,\n      "size": 0,\n      "sha256": "%s"\n    }\n  ]\n}' % SHA, None),
    ("unknown_fields_skipped", base(extra='{"a": [1, -2.5e-3, true, false, null, "x\\n", {}], "b": []}'), None),
    ("options_null", base(parity_shards="null", shard_size="null", plaintext_size="null"), None),
    ("field_order_free", '{"chunks": [], "chunk_count": 0, "chunk_size": 1, "total_size": 0, "version": 1}', None),
    ("escaped_key_and_value", base(**{"versio\\u006e": "3", "version": None}), None),
    ("kind_map_form", chunk(kind='{"parity": null}'), None),
    ("kind_data_explicit", chunk(kind='"data"'), None),
    ("seq_form", '[1, 10, 10, 1, [[0, 10, "%s"]]]' % SHA, None),
    ("seq_form_all_options", '[1, 10, 10, 1, [[0, 10, "%s", "parity"]], 2, 10, null]' % SHA, None),
    ("depth_127_ok", base(extra="[" * 126 + "]" * 126), None),
    ("u64_max", base(total_size="18446744073709551615"), None),
    ("u32_max", base(chunk_count="4294967295"), None),
    # -- rejected ------------------------------------------------------------
    ("missing_version", base(version=None), "missing field `version`"),
    ("missing_total_size", base(total_size=None), "missing field `total_size`"),
    ("missing_chunk_size", base(chunk_size=None), "missing field `chunk_size`"),
    ("missing_chunk_count", base(chunk_count=None), "missing field `chunk_count`"),
    ("missing_chunks", base(chunks=None), "missing field `chunks`"),
    ("missing_index", chunk(index=None), "missing field `index`"),
    ("missing_size", chunk(size=None), "missing field `size`"),
    ("missing_sha256", chunk(sha256=None), "missing field `sha256`"),
    ("empty_object", "{}", "missing field `version`"),
    ("kind_unknown", chunk(kind='"foo"'), "unknown variant `foo`"),
    ("kind_capitalised", chunk(kind='"Parity"'), "unknown variant `Parity`"),
    ("kind_number", chunk(kind="1"), "invalid type"),
    ("kind_null", chunk(kind="null"), "invalid type: null"),
    ("kind_map_value", chunk(kind='{"parity": 1}'), "expected unit"),
    ("version_u32_overflow", base(version="4294967296"), "invalid value: integer `4294967296`, expected u32"),
    ("index_u32_overflow", chunk(index="4294967296"), "expected u32"),
    ("parity_shards_u32_overflow", base(parity_shards="4294967296"), "expected u32"),
    ("total_size_u64_overflow", base(total_size="18446744073709551616"), "floating point"),
    ("negative", base(chunk_count="-1"), "invalid value: integer `-1`"),
    ("negative_zero", base(chunk_count="-0"), "floating point"),
    ("float", base(chunk_size="10.0"), "invalid type: floating point `10.0`"),
    ("exponent", chunk(size="1e3"), "floating point"),
    ("leading_zero", base(total_size="010"), "invalid number"),
    ("plus_sign", base(total_size="+10"), "expected value"),
    ("string_number", base(total_size='"10"'), "invalid type: string"),
    ("null_required", base(version="null"), "invalid type: null"),
    ("bool_number", base(version="true"), "invalid type: boolean"),
    ("sha_number", chunk(sha256="5"), "expected a string"),
    ("chunks_object", base(chunks="{}"), "expected a sequence"),
    ("duplicate_field", base(extra=None) [:-1] + ', "version": 1}', "duplicate field `version`"),
    ("duplicate_chunk_field", chunk(size="10, \"size\": 11"), "duplicate field `size`"),
    ("trailing_comma_object", base()[:-1] + ",}", "trailing comma"),
    ("trailing_comma_array", base(chunks="[" + CHUNK + ",]"), "trailing comma"),
    ("trailing_characters", base() + " x", "trailing characters"),
    ("two_documents", base() + base(), "trailing characters"),
    ("lone_surrogate", chunk(sha256='"\\ud800"'), "hex escape"),
    ("lone_trailing_surrogate", chunk(sha256='"\\udc00"'), "surrogate"),
    ("bad_escape", chunk(sha256='"\\x41"'), "invalid escape"),
    ("raw_control_char", chunk(sha256='"a\tb"'), "control character"),
    ("depth_128", base(extra="[" * 127 + "]" * 127), "recursion limit exceeded"),
    ("deep_nesting", base(extra="[" * 100000 + "]" * 100000), "recursion limit exceeded"),
    ("form_feed_whitespace", "\f" + base(), "expected value"),
    ("unterminated", base()[:-1], "EOF"),
    ("unquoted_key", '{version: 1}', "key must be a string"),
    ("missing_colon", '{"version" 1}', "expected `:`"),
    ("top_level_string", '"manifest"', "invalid type: string"),
    ("empty_input", "", "EOF while parsing a value"),
    ("seq_too_short", "[1, 10]", "invalid length 2"),
    ("seq_too_long", '[1, 10, 10, 1, [], 2, 10, 5, 9]', "trailing characters"),
    ("nan", base(total_size="NaN"), "expected value"),
]


@pytest.fixture(scope="module")
def tools(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("san")
    mc = str(d / "manifest_check")
    oc = str(d / "oracle_check")
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", *SAN, "-o", mc,
                    os.path.join(HERE, "manifest_check.cpp"), os.path.join(ROOT, "maxio_amd", "csrc", "manifest.cpp")],
                   check=True)
    osrc = [os.path.join(ROOT, "oracle", f) for f in ("rs_oracle.c", "sha256_oracle.c", "body_oracle.c", "gcm_oracle.c")]
    subprocess.run(["gcc", "-std=c11", "-Wall", *SAN, "-o", oc, os.path.join(HERE, "oracle_check.c"), *osrc],
                   check=True)
    return mc, oc, d


def run_cases(mc, d, cases):
    files = []
    for name, text, _ in cases:
        p = d / f"{name}.json"
        p.write_bytes(text if isinstance(text, bytes) else text.encode())
        files.append(str(p))
    r = subprocess.run([mc, *files], capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return [json.loads(line) for line in r.stdout.splitlines()]


def test_malformed_manifests_rejected_like_serde(tools):
    mc, _, d = tools
    out = run_cases(mc, d, CASES)
    assert len(out) == len(CASES)
    for (name, _, want), got in zip(CASES, out):
        if want is None:
            assert got["ok"], (name, got)
        else:
            assert not got["ok"], (name, got)
            assert want in got["error"], (name, want, got["error"])


def test_accepted_values(tools):
    mc, _, d = tools
    out = {o["file"].rsplit("/", 1)[1][:-5]: o for o in run_cases(mc, d, [c for c in CASES if c[2] is None])}
    v = out["valid_v2"]
    assert (v["version"], v["total_size"], v["chunk_size"], v["chunk_count"]) == (2, 10, 10, 1)
    assert v["kinds"] == "DP" and v["index"] == [0, 1] and v["sha256"] == [SHA, SHA]
    assert v["parity_shards"] == 1 and v["shard_size"] == 10 and v["plaintext_size"] is None
    assert out["options_null"]["parity_shards"] is None and out["options_null"]["shard_size"] is None
    assert out["escaped_key_and_value"]["version"] == 3
    assert out["kind_map_form"]["kinds"] == "P" and out["kind_data_explicit"]["kinds"] == "D"
    s = out["seq_form_all_options"]
    assert s["kinds"] == "P" and s["parity_shards"] == 2 and s["shard_size"] == 10 and s["plaintext_size"] is None
    assert out["u64_max"]["total_size"] == 2 ** 64 - 1 and out["u32_max"]["chunk_count"] == 2 ** 32 - 1


def test_unicode_escapes_decoded(tools):
    mc, _, d = tools
    esc = "".join("\\u%04x" % ord(c) for c in SHA)
    cases = [("u_escape_sha", chunk(sha256=f'"{esc}"'), None),
             ("surrogate_pair", chunk(sha256='"\\ud83d\\ude00"'), None),
             ("utf8_raw", chunk(sha256='"é"'), None)]
    out = run_cases(mc, d, cases)
    assert out[0]["sha256"] == [SHA]
    assert out[1]["sha256"] == ["\U0001F600"]
    assert out[2]["sha256"] == ["é"]


def test_invalid_utf8_is_an_io_error(tools):
    mc, _, d = tools
    for name, raw in (("latin1", base().replace(SHA, "\xe9" * 64).encode("latin-1")),
                      ("overlong", base().encode().replace(b'"ab', b'"\xc0\xaf')),
                      ("surrogate_bytes", base().encode().replace(b'"ab', b'"\xed\xa0\x80'))):
        out = run_cases(mc, d, [(name, raw, "x")])
        assert out[0]["ok"] is False and out[0].get("io") is True, (name, out)


def test_writer_reader_roundtrip_sanitized(tools):
    mc, _, _ = tools
    r = subprocess.run([mc, "--roundtrip"], capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0 and '"failed": 0' in r.stdout, r.stdout + r.stderr[-2000:]


def test_oracle_under_sanitizers(tools):
    _, oc, _ = tools
    r = subprocess.run([oc], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0 and "oracle_check ok" in r.stdout, r.stdout + r.stderr[-3000:]


def _python_verdict(text: bytes):
    """Syntax per Python's json (RFC 8259 plus NaN / Infinity, which the
    reader rejects): True accepted, False rejected, None no verdict."""
    try:
        s = text.decode("utf-8")
    except UnicodeDecodeError:
        return None
    if "NaN" in s or "Infinity" in s:
        return None
    try:
        json.loads(s)
        return True
    except RecursionError:
        return None
    except ValueError:
        return False


KNOWN = ("version", "total_size", "chunk_size", "chunk_count", "parity_shards", "shard_size", "plaintext_size")


def test_fuzzed_manifests_no_crash_and_consistent_with_json(tools):
    """3 000 mutants of the CASES (byte flips, deletions, insertions of JSON
    punctuation, truncations) through the sanitized reader: no sanitizer
    report, one verdict per input, every input Python's json rejects as JSON
    is rejected too, and every accepted input is valid JSON whose fields are
    the reader's values (map form)."""
    import random

    mc, _, d = tools
    rnd = random.Random(0x6D6178)
    seeds = [c[1].encode() if isinstance(c[1], str) else c[1] for c in CASES if len(c[1]) < 4000]
    tokens = [b"{", b"}", b"[", b"]", b",", b":", b'"', b"\\", b"0", b"-", b"e", b"null", b"true", b"1.5",
              b'"kind"', b'"parity"', b"\\u00", b" ", b"\n", b"\x00", b"\xff"]
    cases = []
    for i in range(3000):
        t = bytearray(rnd.choice(seeds))
        for _ in range(rnd.randint(1, 4)):
            op = rnd.randrange(4)
            pos = rnd.randrange(len(t) + 1)
            if op == 0 and t:
                t[min(pos, len(t) - 1)] ^= 1 << rnd.randrange(8)
            elif op == 1 and t:
                del t[min(pos, len(t) - 1): min(pos, len(t) - 1) + rnd.randint(1, 8)]
            elif op == 2:
                t[pos:pos] = rnd.choice(tokens)
            else:
                t = t[:pos]
        cases.append((f"fz{i}", bytes(t), None))
    out = run_cases(mc, d, cases)
    assert len(out) == len(cases)
    accepted = 0
    for (name, raw, _), got in zip(cases, out):
        verdict = _python_verdict(raw)
        if verdict is False:
            assert not got["ok"], (name, raw[:200], got)
        if got["ok"]:
            accepted += 1
            assert verdict is not False, (name, raw[:200])
            v = json.loads(raw.decode())
            if isinstance(v, dict):
                for f in KNOWN:
                    if f in got and f in v:
                        assert got[f] == v[f], (name, f, got[f], v[f])
    assert accepted > 50  # the mutants do exercise the accepting paths
