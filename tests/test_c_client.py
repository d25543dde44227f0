"""The C ABI from a plain C99 program (tests/c_client/put_get.c), the way
MaxIO's extern "C" block would call it: compiled with gcc against
include/maxio_ec.h and linked to libmaxio_ec.so (CPU), then run on the GPU:
BASELINE configs[0] (10 MiB PUT, delete shard 000000, GET) and a bitrot /
lost-parity / ranged-GET object, ending with the too-many-missing error."""
from __future__ import annotations

import os
import subprocess

import pytest

import maxio_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    exe = tmp_path / "put_get"
    lib_dir = os.path.dirname(maxio_amd.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-D_POSIX_C_SOURCE=200809L", "-O2", "-Wall", "-Werror",
                    os.path.join(ROOT, "tests", "c_client", "put_get.c"),
                    "-I", os.path.join(ROOT, "include"), "-L", lib_dir, "-lmaxio_ec",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True)
    return exe


def test_c_client_builds_and_links(tmp_path):
    exe = _build(tmp_path)
    assert exe.exists()


@pytest.mark.gpu
def test_c_client_put_get_roundtrip(tmp_path):
    exe = _build(tmp_path)
    scratch = tmp_path / "data"
    scratch.mkdir()
    r = subprocess.run([str(exe), str(scratch)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "c client ok" in r.stdout
