#!/usr/bin/env python3
"""The SDMA watch on the verified GET (pipeline.cpp watch_open / watch_judge):
what its upload brackets read in a fresh process, next to the same batch
with every copy forced to SDMA and to waves.

128 x 4+2 x 10 MiB from mxec_host_alloc memory, two erasures per object;
one PUT with digests, then per copy mode (auto, sdma, waves; a context each)
a warm GET and `--reps` timed verified GETs, each with its pipeline-counter
deltas (checks, slow verdicts, the last bracket's rate, wave blocks).  One
JSON line per mode.

  python tools/watch_diag.py [--objects 128] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (the process's HIP runtime, as in bench.py)

    import maxio_amd

    k, m, S, n = 4, 2, 10 << 20, a.objects
    rng = np.random.default_rng(5)
    base = maxio_amd.Context(streams_per_device=2)
    buf = base.host_array(n * (k + m) * S).reshape(n, k + m, S)
    blk = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    flat = buf.reshape(-1)
    for o in range(0, flat.size, blk.size):
        flat[o:o + min(blk.size, flat.size - o)] = blk[:min(blk.size, flat.size - o)] ^ np.uint8(o >> 26)
    objs = [(k, m, S)] * n
    dig = np.zeros(n * (k + m) * 32, np.uint8)
    base.encode_batch_host(objs, [buf[o, j].ctypes.data for o in range(n) for j in range(k)],
                           [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)], digests=dig)
    present0 = np.ones(n * (k + m), np.uint8)
    for o in range(n):
        for i in rng.choice(k + m, 2, replace=False):
            present0[o * (k + m) + i] = 0
    sptr = [buf[o, i].ctypes.data for o in range(n) for i in range(k + m)]
    for mode in ("auto", "sdma", "waves"):
        os.environ["MXEC_PIPE_COPY"] = mode
        ctx = maxio_amd.Context(streams_per_device=2)
        os.environ.pop("MXEC_PIPE_COPY")
        row = {"mode": mode, "objects": n, "calls": []}
        for rep in range(a.reps + 1):
            s0 = ctx.pipe_stats()
            pr = present0.copy()
            t0 = time.perf_counter()
            rc, st = ctx.reconstruct_batch_host(objs, sptr, pr, expected=dig)
            el = time.perf_counter() - t0
            s1 = ctx.pipe_stats()
            assert rc == 0 and not st.any()
            row["calls"].append({"s": round(el, 4), "warm": rep == 0,
                                 **{key: s1[key] - s0[key] for key in ("sdma_checks", "sdma_slow", "wave_blocks",
                                                                      "copies_1d")},
                                 "sdma_last_mbps": s1["sdma_last_mbps"]})
        ctx.close()
        print(json.dumps(row), flush=True)
    base.host_free(buf)
    base.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
