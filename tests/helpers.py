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
