"""Data generators shared by tests and tests/golden/make_golden.py."""
from __future__ import annotations

import numpy as np

SEED = 0x6D6178696F  # "maxio"


def data_for(seed: int, k: int, size: int, last: int | None = None) -> list[np.ndarray]:
    rng = np.random.default_rng(seed)
    out = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    if last is not None:
        out[-1] = out[-1][:last].copy()
    return out


def scenario_body(spec: dict) -> bytes:
    unit = bytes.fromhex(spec["unit_hex"])
    n = spec["len"]
    return (unit * (n // max(1, len(unit)) + 1))[:n] if n else b""


def sha_vector_inputs(seed: int, lens: list[int]) -> list[bytes]:
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]


def expected_ec_object(stream: bytes, chunk_size: int, m: int, plaintext_size=None):
    """The files and manifest.json text filesystem.rs writes for `stream`
    (put_object_chunked :686-828 and the encrypted / multipart drivers that
    chunk a stream the same way): {name: bytes}, manifest text.  Parity from
    the oracle (crate algorithm), digests from hashlib, manifest in
    serde_json::to_string_pretty layout."""
    import hashlib
    import json

    import oracle

    data = [stream[o:o + chunk_size] for o in range(0, len(stream), chunk_size)] or [b""]
    has_parity = m > 0 and len(stream) > 0
    files = {f"{j:06}": d for j, d in enumerate(data)}
    chunks = [{"index": j, "size": len(d), "sha256": hashlib.sha256(d).hexdigest()} for j, d in enumerate(data)]
    if has_parity:
        parity = oracle.encode([np.frombuffer(d, np.uint8) for d in data], m, chunk_size)
        for i, p in enumerate(parity):
            b = p.tobytes()
            files[f"{len(data) + i:06}"] = b
            chunks.append({"index": len(data) + i, "size": chunk_size,
                           "sha256": hashlib.sha256(b).hexdigest(), "kind": "parity"})
    man = {"version": 2 if has_parity else 1, "total_size": len(stream), "chunk_size": chunk_size,
           "chunk_count": len(data), "chunks": chunks}
    if has_parity:
        man["parity_shards"] = m
        man["shard_size"] = chunk_size
    if plaintext_size is not None:
        man["plaintext_size"] = plaintext_size
    return files, json.dumps(man, indent=2)
