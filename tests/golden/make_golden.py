"""Generate the committed golden fixtures under tests/golden/.

Run: python tests/golden/make_golden.py

Sources of truth (nothing from /root/reference is copied or executed):
  * reed-solomon-erasure 6.0.0 published known answers, restated by hand in
    rs_kat.json: galois_8 `mul`, `div`, `exp` test values and the
    `test_one_encode` 5+5 vector.
  * SHA-256: Python hashlib (OpenSSL) and the FIPS 180-4 empty-string digest.
  * Encode / reconstruct vectors: oracle/ (the C restatement, itself pinned by
    the known answers above in tests/test_oracle.py); data regenerated from
    numpy PCG64 seeds, so only seeds and output digests are stored.
  * Reference scenarios (tests/integration.rs:3155-3385): file layout and the
    manifest as serde_json::to_string_pretty writes it — json.dumps(indent=2)
    produces the same bytes for this schema (two-space indent, ": " and ",").
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

SEED = 0x6D6178696F  # "maxio"


def data_for(seed: int, k: int, size: int, last: int | None = None) -> list[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    if last is not None:
        out[-1] = out[-1][:last].copy()
    return out


def rs_kat() -> dict:
    return {
        "source": "reed-solomon-erasure 6.0.0 galois_8 tests + core test_one_encode",
        "gf_mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
        "gf_div": [[0, 7, 0], [3, 3, 1], [6, 3, 2]],
        "gf_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
        "one_encode": {
            "k": 5, "m": 5,
            "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
            "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]],
        },
        "parity_rows": {
            f"{k}+{m}": oracle.matrix(k, m)[k:].tolist()
            for (k, m) in [(1, 2), (4, 2), (8, 4), (10, 4), (5, 5), (64, 4)]
        },
    }


def encode_vectors() -> dict:
    cases = []
    n = 0
    for (k, m) in [(1, 2), (4, 2), (8, 4), (10, 4)]:
        for size in [100, 1024, 4096]:
            for last in [None, size // 2 + 3]:
                seed = SEED ^ n
                n += 1
                data = data_for(seed, k, size, last)
                parity, digests, rc = oracle.compute_parity(data, m, size)
                assert rc == 0
                cases.append({
                    "k": k, "m": m, "shard_size": size, "seed": seed,
                    "last_len": last if last is not None else size,
                    "parity_sha256": [hashlib.sha256(p.tobytes()).hexdigest() for p in parity],
                    "parity_head": [p[:16].tobytes().hex() for p in parity],
                    "chunk_sha256": [d.hex() for d in digests],
                })
    return {"generator": "oracle.compute_parity (filesystem.rs:1084-1145 restated)", "cases": cases}


def reconstruct_vectors() -> dict:
    import itertools

    cases = []
    for (k, m, size) in [(4, 2, 100), (8, 4, 64)]:
        seed = SEED ^ (k << 8 | m)
        data = data_for(seed, k, size)
        parity = oracle.encode(data, m, size)
        shards = data + parity
        patterns = [list(p) for e in (1, 2) for p in itertools.combinations(range(k + m), e)]
        for pat in patterns:
            inp = [None if i in pat else shards[i] for i in range(k + m)]
            out, present, rc = oracle.reconstruct(inp, k, m, size)
            assert rc == 0 and all(np.array_equal(out[i], shards[i]) for i in range(k + m))
        cases.append({
            "k": k, "m": m, "shard_size": size, "seed": seed, "erasure_patterns": patterns,
            "shard_sha256": [hashlib.sha256(s.tobytes()).hexdigest() for s in shards],
        })
    return {"generator": "oracle.reconstruct (crate reconstruct_internal restated)", "cases": cases}


def sha_vectors() -> dict:
    rng = np.random.default_rng(SEED)
    out = []
    for n in [0, 1, 55, 56, 63, 64, 65, 100, 119, 120, 1024, 1 << 20]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out.append({"len": n, "seed_order": len(out), "sha256": hashlib.sha256(b).hexdigest()})
    return {
        "generator": "hashlib.sha256 over numpy default_rng(SEED) integers, lengths in order",
        "seed": SEED,
        "empty": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        "cases": out,
    }


def manifest_text(chunks: list[dict], total: int, chunk_size: int, m: int) -> str:
    has_parity = m > 0 and total > 0
    man = {
        "version": 2 if has_parity else 1,
        "total_size": total,
        "chunk_size": chunk_size,
        "chunk_count": sum(1 for c in chunks if c.get("kind") != "parity"),
        "chunks": chunks,
    }
    if has_parity:
        man["parity_shards"] = m
        man["shard_size"] = chunk_size
    return json.dumps(man, indent=2)


def scenario(unit: bytes, length: int, chunk_size: int, m: int) -> dict:
    body = (unit * (length // max(1, len(unit)) + 1))[:length] if length else b""
    data = [np.frombuffer(body[o:o + chunk_size], np.uint8) for o in range(0, len(body), chunk_size)]
    if not data:
        data = [np.zeros(0, np.uint8)]
    has_parity = m > 0 and len(body) > 0
    files, chunks = {}, []
    for j, d in enumerate(data):
        files[f"{j:06}"] = {"size": int(d.size)}
        chunks.append({"index": j, "size": int(d.size), "sha256": hashlib.sha256(d.tobytes()).hexdigest()})
    if has_parity:
        parity, digests, rc = oracle.compute_parity(data, m, chunk_size)
        assert rc == 0
        for i, p in enumerate(parity):
            idx = len(data) + i
            files[f"{idx:06}"] = {"size": chunk_size, "hex": p.tobytes().hex()}
            chunks.append({"index": idx, "size": chunk_size, "sha256": digests[idx].hex(), "kind": "parity"})
    return {"chunk_size": chunk_size, "parity_shards": m,
            "body": {"unit_hex": unit.hex(), "len": length}, "files": files,
            "manifest": manifest_text(chunks, len(body), chunk_size, m)}


def reference_scenarios() -> dict:
    per_chunk = b"".join(bytes([i + 1]) * (100 if i < 3 else 50) for i in range(4))
    return {
        "source": "tests/integration.rs parity scenarios, replayed at the byte level",
        "parity_write_0xAB_350": scenario(b"\xab", 350, 100, 2),      # :3155
        "parity_read_0xCD_350": scenario(b"\xcd", 350, 100, 2),       # :3194
        "parity_corrupt_0xEF_350": scenario(b"\xef", 350, 100, 2),    # :3214
        "parity_missing_0x42_350": scenario(b"\x42", 350, 100, 2),    # :3239
        "parity_too_many_0x77_350": scenario(b"\x77", 350, 100, 2),   # :3263
        "parity_range_per_chunk_350": scenario(per_chunk, 350, 100, 2),  # :3299
        "v1_no_parity_0xAA_2048": scenario(b"\xaa", 2048, 1024, 0),   # :3336
        "empty_with_parity": scenario(b"", 0, 100, 2),                 # :3357
        "ec_put_get_0x42_3072": scenario(b"\x42", 3072, 1024, 0),     # :2702
        "ec_plus_parity_k49": scenario(bytes(range(256)), 50000, 1024, 2),  # :5646 (k=49)
    }


def main() -> None:
    outputs = {
        "rs_kat.json": rs_kat(),
        "encode_vectors.json": encode_vectors(),
        "reconstruct_vectors.json": reconstruct_vectors(),
        "sha256_vectors.json": sha_vectors(),
        "reference_scenarios.json": reference_scenarios(),
    }
    for name, obj in outputs.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")
        print(name, os.path.getsize(os.path.join(HERE, name)))


if __name__ == "__main__":
    main()
