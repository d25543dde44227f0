#!/usr/bin/env python3
"""Lane-level model of the SHA-256 "lag" quad form (sha256_kernel.hip,
compress_lag), checked against hashlib.

The quad form runs the e-side and the a-side of a round as ONE instruction
stream in two lanes of a quad (lane E: e, f, g, h; lane A: a, b, c, d).  In
the first version both lanes work on the same round t, so lane A's
a' = T1 + T2 needs lane E's T1 of that very round: a DPP add sits on every
round's critical path.  Here lane A runs two rounds behind lane E:

  step t, lane E:  e[t+1] = Σ1(e[t]) + Ch(e[t], e[t-1], e[t-2]) + H
                   H = e[t-3] + a[t-3] + K[t] + W[t]          (h + d + K + W)
  step t, lane A:  a[t-1] = Σ0(a[t-2]) + Maj(a[t-2], a[t-3], a[t-4]) + H
                   H = T1[t-2] = e[t-1] - a[t-5]

Both lanes read the OTHER lane's "X1" register (the value written one step
earlier: a[t-3] in lane A, e[t-1] in lane E) through one DPP swap, so the
only cross-lane operand is a step old, and a step is

  3 x v_alignbit, v_bitop3 (xor3), v_bitop3 (selector), v_bitop3 (Ch),
  v_xad (X3 ^ mask + c), v_add_dpp (+ other lane's X1), v_add3   = 9 VALU

with X -> alignbit -> xor3 -> add3 -> X' the chain.  A block takes 66
steps (lane A's last two rounds run while lane E computes two unused
values), lane A's first two outputs are forced to the known b and a.
History is an 8-register ring x[t & 7]; lane A keeps its state rotated as
(c, d, a, b) so that both lanes load and most of them store the same ring
slots.

  python tools/sha_lag_model.py      # random messages vs hashlib
"""
from __future__ import annotations

import hashlib
import os
import struct

M32 = 0xFFFFFFFF
K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & M32


def kw_words(block: bytes) -> list[int]:
    """The producer's K[t] + W[t] of one 64-byte block."""
    w = list(struct.unpack(">16I", block))
    for t in range(16, 64):
        s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)
        s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & M32)
    return [(K[t] + w[t]) & M32 for t in range(64)]


E, A = 0, 1
SH = {E: (6, 11, 25), A: (2, 13, 22)}
MA = {E: 0, A: M32}


def compress_lag(s: dict[int, list[int]], kw: list[int]) -> None:
    """One block on the two lanes of a message, as the kernel's instruction
    stream does it (every lane executes every step)."""
    x = {r: [0] * 8 for r in (E, A)}
    for r in (E, A):
        x[r][0], x[r][7], x[r][6], x[r][5] = s[r][0], s[r][1], s[r][2], s[r][3]
    for t in range(66):
        # reads of the step (the DPP reads the other lane's X1, written a step ago)
        X = {r: (x[r][t & 7], x[r][(t - 1) & 7], x[r][(t - 2) & 7], x[r][(t - 3) & 7]) for r in (E, A)}
        out = {}
        for r in (E, A):
            X0, X1, X2, X3 = X[r]
            a1, a2, a3 = SH[r]
            S = rotr(X0, a1) ^ rotr(X0, a2) ^ rotr(X0, a3)
            sel = X0 ^ (~X1 & MA[r] & M32)
            ch = (sel & X1) | (~sel & M32 & X2)
            c = (kw[t] if t < 64 else 0) if r == E else 1
            t1 = ((X3 ^ MA[r]) + c) & M32
            H = (X[1 - r][1] + t1) & M32
            P = (S + ch + H) & M32
            if r == A and t == 0:
                P = s[A][3]  # b
            if r == A and t == 1:
                P = s[A][2]  # a
            out[r] = P
        for r in (E, A):
            x[r][(t + 1) & 7] = out[r]
    s[E][0] = (s[E][0] + x[E][0]) & M32
    s[E][1] = (s[E][1] + x[E][7]) & M32
    s[E][2] = (s[E][2] + x[E][6]) & M32
    s[E][3] = (s[E][3] + x[E][5]) & M32
    s[A][0] = (s[A][0] + x[A][0]) & M32
    s[A][1] = (s[A][1] + x[A][7]) & M32
    s[A][2] = (s[A][2] + x[A][2]) & M32
    s[A][3] = (s[A][3] + x[A][1]) & M32


def sha256_lag(msg: bytes) -> bytes:
    n = len(msg)
    padded = msg + b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
    a, b, c, d, e, f, g, h = IV
    s = {E: [e, f, g, h], A: [c, d, a, b]}
    for o in range(0, len(padded), 64):
        compress_lag(s, kw_words(padded[o:o + 64]))
    c, d, a, b = s[A]
    e, f, g, h = s[E]
    return struct.pack(">8I", a, b, c, d, e, f, g, h)


def main() -> None:
    rng = os.urandom
    for n in [0, 1, 55, 56, 63, 64, 65, 119, 128, 1000, 4096 + 7]:
        m = rng(n)
        assert sha256_lag(m) == hashlib.sha256(m).digest(), n
    print("lag model == hashlib for 11 lengths")


if __name__ == "__main__":
    main()
