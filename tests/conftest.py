"""Shared fixtures.  `-m gpu` tests need an MI355X and the built
libmaxio_ec.so; everything else runs on CPU."""
from __future__ import annotations

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's): whichever
# loads first serves the whole process.  Load torch's first so the tests that
# use torch as a device allocator and libmaxio_ec share that runtime, as in
# bench.py.
try:
    import torch  # noqa: F401
except ImportError:  # CPU-only environments without torch still run the oracle tests
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libmaxio_ec.so")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name: str):
        if name not in cache:
            with open(os.path.join(GOLDEN, name)) as f:
                cache[name] = json.load(f)
        return cache[name]

    return load


@pytest.fixture(scope="session")
def ctx():
    import maxio_amd

    c = maxio_amd.Context(streams_per_device=2)
    yield c
    c.close()
