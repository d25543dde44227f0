"""CPU: the C-ABI library loads, exports every symbol include/maxio_ec.h
declares, is plain C, and its host-side matrix algebra equals the oracle.
No kernel is launched here."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import maxio_amd
import oracle
from maxio_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    lib = maxio_amd.lib()
    declared = maxio_amd.declared_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", maxio_amd.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\b(mxec_\w+)$", out, re.M))
    assert set(declared) == exported


def test_header_is_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "maxio_ec.h"\nint main(void){ return mxec_rs_check(4, 2); }\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", str(src), "-I",
                    os.path.join(ROOT, "include"), "-o", str(tmp_path / "t.o")], check=True)


def test_rs_check_matches_crate():
    for k in [0, 1, 2, 128, 200, 255, 256]:
        for m in [0, 1, 2, 56, 57, 128]:
            assert maxio_amd.lib().mxec_rs_check(k, m) == oracle.rs_check(k, m), (k, m)


@pytest.mark.parametrize("k,m", [(1, 2), (4, 2), (5, 5), (8, 4), (10, 4), (64, 4), (17, 9),
                                 (128, 127), (253, 2), (1, 254)])
def test_parity_matrix_matches_oracle(k, m):
    assert np.array_equal(maxio_amd.parity_matrix(k, m), oracle.matrix(k, m)[k:])


def test_rs_check_raises_named_errors():
    with pytest.raises(maxio_amd.RSError) as e:
        maxio_amd.rs_check(4, 0)
    assert e.value.name == "TooFewParityShards"
    with pytest.raises(maxio_amd.RSError) as e:
        maxio_amd.rs_check(0, 4)
    assert e.value.name == "TooFewDataShards"


def test_strerror_and_version():
    lib = maxio_amd.lib()
    assert b"gfx950" in lib.mxec_version()
    for code in [0, -1, -10, -20, -30, -40]:
        assert lib.mxec_strerror(code)


def test_open_without_gpu_fails_loudly():
    if maxio_amd.device_count() > 0:
        pytest.skip("a HIP device is visible")
    assert maxio_amd.lib().mxec_open(0, 1) is None
    assert b"no HIP device" in maxio_amd.lib().mxec_last_error()
    with pytest.raises(maxio_amd.RSError):
        maxio_amd.Context()


def test_product_never_touches_oracle():
    """The product path may not import, link or call the oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "maxio_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", "Makefile", ".map")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "import oracle" not in text and "liboracle" not in text, f
                assert "orc_" not in text, f
    libs = subprocess.run(["ldd", maxio_amd.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in libs


def test_missing_library_is_loud(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_native.NativeLibraryMissing):
        _native.lib()


def test_chunk_info_layout():
    # mxec_chunk_info: u32 index, u64 size, char[65], u8 kind
    assert ctypes.sizeof(_native.ChunkInfo) == 8 + 8 + 65 + 1 + 6
