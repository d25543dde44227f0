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


TEST_OPTIONS = {"MXEC_TEST_LOGICAL_DEVICES": "logical_devices", "MXEC_TEST_RS_GRID": "rs_grid",
                "MXEC_TEST_COEF_ARENA_KB": "coef_arena_kb"}


def open_ctx(streams=2, device_mask=0, **env):
    """A context opened with MXEC_* settings: the library reads its knobs
    once, at mxec_open (maxio_amd/csrc/knobs.cpp), so a test that changes
    one opens its own context.  Values None / "" unset the variable.  The
    MXEC_TEST_* names are not environment variables: they become
    mxec_open_test arguments (Context(test=...))."""
    import maxio_amd

    test = {TEST_OPTIONS[k]: int(env.pop(k)) for k in list(env) if k in TEST_OPTIONS}
    saved = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            if v is None or v == "":
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        return maxio_amd.Context(device_mask=device_mask, streams_per_device=streams, test=test or None)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="session")
def ctx_with():
    """Session cache of open_ctx contexts, one per distinct setting:
    ctx_with(streams=2, MXEC_X="1")."""
    cache = {}

    def get(streams=2, device_mask=0, **env):
        key = (streams, device_mask, tuple(sorted((k, str(v)) for k, v in env.items())))
        if key not in cache:
            cache[key] = open_ctx(streams, device_mask, **env)
        return cache[key]

    yield get
    for c in cache.values():
        c.close()


def lab_build() -> bool:
    """True when the loaded library is the lab build (make lab; MXEC_LIB)."""
    import maxio_amd

    return "lab build" in maxio_amd.version()
