#!/usr/bin/env python3
"""Within-process A/B of the host PUT pipeline with digests
(mxec_encode_batch_host from page-locked memory, RS + SHA-256 of every
chunk): MXEC_PIPE_PIECE_MB values alternate round by round (0 = the group
form, n = piece-major with n MiB pieces), wall clock per batch; parity and
digests compared across arms, one chunk's digest against hashlib.  Lab
tool, not product.

  python tools/e2e_piece_ab.py [--objects 128] [--values 0,1,2] [--rounds 3] [--get]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# The lab knobs exist only in the lab build (make -C maxio_amd/csrc lab).
os.environ.setdefault("MXEC_LIB", os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--chunk-size", type=int, default=10 << 20)
    ap.add_argument("--env", default="MXEC_PIPE_PIECE_MB",
                    help="the knob alternated (one context per value: knobs are read at mxec_open)")
    ap.add_argument("--values", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-digests", action="store_true")
    ap.add_argument("--get", action="store_true", help="also A/B the verified GET (2 erasures per object)")
    a = ap.parse_args()
    import numpy as np

    import maxio_amd

    k, m, S, n = 4, 2, a.chunk_size, a.objects
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    data = ctx.host_array(n * k * S).reshape(n, k, S)
    par = ctx.host_array(n * m * S).reshape(n, m, S)
    rng = np.random.default_rng(5)
    for o in range(n):
        data[o] = rng.integers(0, 256, (k, S), dtype=np.uint8)
    dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
    pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
    objs = [(k, m, S)] * n
    ctxs = {}
    for v in a.values.split(","):
        os.environ[a.env] = v
        ctxs[v] = maxio_amd.Context(device_mask=1, streams_per_device=2)
    seen = {}
    for rnd in range(a.rounds):
        for v in a.values.split(","):
            c = ctxs[v]
            dig = None if a.no_digests else np.zeros(n * (k + m) * 32, np.uint8)
            c.encode_batch_host(objs, dptr, pptr, digests=dig)  # warm
            t0 = time.perf_counter()
            c.encode_batch_host(objs, dptr, pptr, digests=dig)
            el = time.perf_counter() - t0
            snap = (par[n // 2].copy(), None if dig is None else dig.copy())
            if v in seen:
                assert np.array_equal(seen[v][0], snap[0])
            seen[v] = snap
            print(json.dumps({"round": rnd, a.env: v, "s_per_batch": round(el, 4),
                              "GiBps_payload": round(n * k * S / el / 2**30, 2)}), flush=True)
    if a.get and not a.no_digests:
        # GET side: two seeded erasures per object, verified against the
        # digests just computed (mxec_reconstruct_batch_host).
        exp = seen[a.values.split(",")[0]][1]
        sptr = []
        for o in range(n):
            sptr += [data[o, j].ctypes.data for j in range(k)] + [par[o, i].ctypes.data for i in range(m)]
        present0 = np.ones(n * (k + m), np.uint8)
        for o in range(n):
            for i in rng.choice(k + m, 2, replace=False):
                present0[o * (k + m) + i] = 0
        want = par[n // 3].copy(), data[n // 3].copy()
        for rnd in range(a.rounds):
            for v in a.values.split(","):
                c = ctxs[v]
                pr = present0.copy()
                rc, _ = c.reconstruct_batch_host(objs, sptr, pr, expected=exp)  # warm
                assert rc == 0, rc
                pr = present0.copy()
                t0 = time.perf_counter()
                rc, _ = c.reconstruct_batch_host(objs, sptr, pr, expected=exp)
                el = time.perf_counter() - t0
                assert rc == 0 and np.array_equal(par[n // 3], want[0]) and np.array_equal(data[n // 3], want[1])
                print(json.dumps({"get_verify": True, "round": rnd, a.env: v,
                                  "s_per_batch": round(el, 4), "GiBps_payload": round(n * k * S / el / 2**30, 2)}),
                      flush=True)
    arms = list(seen.values())
    same = all(np.array_equal(x[0], arms[0][0]) and (x[1] is None or np.array_equal(x[1], arms[0][1]))
               for x in arms)
    ok = True
    if arms[0][1] is not None:
        o, j = n - 1, k - 1
        ok = hashlib.sha256(data[o, j].tobytes()).digest() == arms[0][1][(o * (k + m) + j) * 32:
                                                                         (o * (k + m) + j + 1) * 32].tobytes()
    print(json.dumps({"equal_across_arms": bool(same), "hashlib_sample_ok": bool(ok)}), flush=True)
    os.environ.pop(a.env, None)
    for c in ctxs.values():
        c.close()
    ctx.close()
    return 0 if same and ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
