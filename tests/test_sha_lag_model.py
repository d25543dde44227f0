"""CPU: the lane-level model of the lag quad SHA-256 form (tools/
sha_lag_model.py: lane E and lane A two rounds apart, one DPP swap of X1 per
step, 66 steps per block) equals hashlib, whole messages and piece by piece
with the chain state carried between pieces as the kernel's piece mode does
(ShaPiece, kernels.hpp).  The model is the design check behind
compress_lag in maxio_amd/csrc/sha256_kernel.hip."""
from __future__ import annotations

import hashlib
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import sha_lag_model as lag  # noqa: E402


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 1000, 4103])
def test_lag_model_matches_hashlib(n):
    m = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert lag.sha256_lag(m) == hashlib.sha256(m).digest()


def _state_to_lanes(st):
    a, b, c, d, e, f, g, h = st
    return {lag.E: [e, f, g, h], lag.A: [c, d, a, b]}


def _lanes_to_state(s):
    c, d, a, b = s[lag.A]
    e, f, g, h = s[lag.E]
    return [a, b, c, d, e, f, g, h]


@pytest.mark.parametrize("piece", [64, 128, 320])
def test_lag_model_in_pieces(piece):
    """Pieces of whole 64-byte blocks, the state (a..h) stored and reloaded
    between them in the kernel's order; the last piece carries the tail and
    pads with the message's total length."""
    n = 1000
    m = np.random.default_rng(piece).integers(0, 256, n, dtype=np.uint8).tobytes()
    padded = m + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
    st = list(lag.IV)
    for o in range(0, len(padded), piece):
        s = _state_to_lanes(st)  # resume: load a..h into the two lanes
        for b in range(o, min(o + piece, len(padded)), 64):
            lag.compress_lag(s, lag.kw_words(padded[b:b + 64]))
        st = _lanes_to_state(s)  # mid-message piece: the state goes back
    assert struct.pack(">8I", *st) == hashlib.sha256(m).digest()
