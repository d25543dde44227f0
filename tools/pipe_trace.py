#!/usr/bin/env python3
"""Timelines of host batch calls (lab build: MXEC_PIPE_TRACE=1, pipeline.cpp
PipeTrace -- one stderr JSON line per wave, GPU marks and host marks against
one process-wide reference, so concurrent calls line up): a PUT with digests
alone, a verified GET alone, and the two started together, 128 x 4+2 x 10 MiB
from page-locked memory (bench.py e2e_concurrent's sets).  Settings via
--env (read at mxec_open).  stdout: one JSON line per phase (its calls' wall
times); the wave lines go to stderr.

  MXEC_LIB=maxio_amd/lib/libmaxio_ec_lab.so python tools/pipe_trace.py --env MXEC_PIPE_COPY=sdma
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MXEC_LIB", os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="")
    ap.add_argument("--objects", type=int, default=128)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401

    import bench
    import maxio_amd

    kv = dict(x.split("=", 1) for x in a.env.split(",") if x)
    os.environ.update(kv)
    ctx = maxio_amd.Context(streams_per_device=2)
    n, k, m, S = a.objects, 4, 2, 10 << 20
    shapes = [(k, m, S)] * n
    put_rows, _, put_d, put_p, _ = bench._encoded_set(ctx, shapes, 31)
    get_rows, get_dig, _, _, _ = bench._encoded_set(ctx, shapes, 32)
    put_dig = np.zeros(n * (k + m) * 32, np.uint8)
    get = bench._GetBatch(ctx, shapes, get_rows, get_dig, 33)

    def put():
        assert (ctx.encode_batch_host(shapes, put_d, put_p, digests=put_dig) == 0).all()

    put(), get.run(), put(), get.run()  # warm
    os.environ["MXEC_PIPE_TRACE"] = "1"
    for phase in ("put", "get", "pair", "pair"):
        print(json.dumps({"phase_start": phase}), file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        ends = {}
        if phase == "pair":
            go = threading.Barrier(2)

            def run(name, fn):
                go.wait()
                fn()
                ends[name] = round(time.perf_counter() - t0, 4)

            th = [threading.Thread(target=run, args=("put", put)), threading.Thread(target=run, args=("get", get.run))]
            for t in th:
                t.start()
            for t in th:
                t.join()
        else:
            (put if phase == "put" else get.run)()
            ends[phase] = round(time.perf_counter() - t0, 4)
        print(json.dumps({"phase": phase, "env": kv, "ends_s": ends, "exact": get.exact()}), flush=True)
        time.sleep(0.2)
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
