#!/usr/bin/env python3
"""Which copy engine should the host batch calls use?  The SDMA watch
(pipeline.cpp watch_open / watch_judge) against the same batches with every
copy forced to SDMA and to CU waves.

Per batch size (`--objects`, 4+2 x 10 MiB from mxec_host_alloc memory, two
erasures per object): one PUT with digests, then per GET kind (verified:
expected digests; rs: none) and copy mode (auto, sdma, waves; a context
each) a warm call and `--reps` timed calls, each with its pipeline-counter
deltas (checks, slow verdicts, the last bracket's rate, wave blocks).
`--churn GB` first allocates and frees that much HBM through torch, as
bench.py's headline does before its host legs; `--churn-each GB` does it
between every warm call and its timed calls (no pause after the free).  One JSON line per
(objects, kind, mode).

  python tools/watch_diag.py [--objects 128,512] [--kinds verified,rs] [--reps 3] [--churn 0]
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
    ap.add_argument("--objects", default="128")
    ap.add_argument("--kinds", default="verified")
    ap.add_argument("--modes", default="auto,sdma,waves")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--churn", type=float, default=0.0)
    ap.add_argument("--churn-each", type=float, default=0.0)
    a = ap.parse_args()
    import numpy as np
    import torch

    import maxio_amd

    def churn(gb: float) -> float:
        t = torch.empty(int(gb * 1e9), dtype=torch.uint8, device="cuda")
        t.fill_(1)
        torch.cuda.synchronize()
        del t
        t0 = time.perf_counter()
        torch.cuda.empty_cache()
        return time.perf_counter() - t0

    if a.churn > 0:
        churn(a.churn)
    k, m, S = 4, 2, 10 << 20
    rng = np.random.default_rng(5)
    base = maxio_amd.Context(streams_per_device=2)
    for n in (int(x) for x in a.objects.split(",")):
        buf = base.host_array(n * (k + m) * S).reshape(n, k + m, S)
        blk = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
        flat = buf.reshape(-1)
        for o in range(0, flat.size, blk.size):
            flat[o:o + min(blk.size, flat.size - o)] = blk[:min(blk.size, flat.size - o)] ^ np.uint8((o >> 26) & 255)
        objs = [(k, m, S)] * n
        dig = np.zeros(n * (k + m) * 32, np.uint8)
        base.encode_batch_host(objs, [buf[o, j].ctypes.data for o in range(n) for j in range(k)],
                               [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)], digests=dig)
        present0 = np.ones(n * (k + m), np.uint8)
        for o in range(n):
            for i in rng.choice(k + m, 2, replace=False):
                present0[o * (k + m) + i] = 0
        sptr = [buf[o, i].ctypes.data for o in range(n) for i in range(k + m)]
        dptr = [buf[o, j].ctypes.data for o in range(n) for j in range(k)]
        pptr = [buf[o, k + i].ctypes.data for o in range(n) for i in range(m)]
        dig2 = np.zeros_like(dig)
        for kind in a.kinds.split(","):
            for mode in a.modes.split(","):
                # sdma_down_waves (lab build): uploads by SDMA, downloads by
                # waves; auto_nowatch: auto with the watch off (floor 0)
                # *_cus16 (lab): copy streams on 16 CUs, compute streams on the rest
                env = {"sdma_down_waves": {"MXEC_PIPE_COPY": "sdma"},
                       "sdma_down_waves_cus16": {"MXEC_PIPE_COPY": "auto", "MXEC_PIPE_SDMA_FLOOR": "0",
                                                 "MXEC_PIPE_COPY_CUS": "16"},
                       "waves_cus16": {"MXEC_PIPE_COPY": "waves", "MXEC_PIPE_COPY_CUS": "16"},
                       "auto_nowatch": {"MXEC_PIPE_COPY": "auto", "MXEC_PIPE_SDMA_FLOOR": "0"}}.get(
                           mode, {"MXEC_PIPE_COPY": mode})
                os.environ.update(env)
                ctx = maxio_amd.Context(streams_per_device=2)
                for key in env:
                    os.environ.pop(key)
                if mode.startswith("sdma_down_waves"):
                    os.environ["MXEC_PIPE_DOWN_WAVES"] = "1"
                else:
                    os.environ.pop("MXEC_PIPE_DOWN_WAVES", None)
                row = {"objects": n, "kind": kind, "mode": mode, "churn_GB": a.churn, "calls": []}
                for rep in range(a.reps + 1):
                    if rep == 1 and a.churn_each > 0:  # after the warm call, right before the timed ones
                        row["free_s"] = round(churn(a.churn_each), 4)
                        row["churn_each_GB"] = a.churn_each
                    s0 = ctx.pipe_stats()
                    pr = present0.copy()
                    t0 = time.perf_counter()
                    if kind.startswith("put"):
                        ctx.encode_batch_host(objs, dptr, pptr, digests=dig2 if kind == "put_sha" else None)
                        rc, st = 0, np.zeros(1, np.uint8)
                    else:
                        rc, st = ctx.reconstruct_batch_host(objs, sptr, pr,
                                                            expected=dig if kind == "verified" else None)
                    el = time.perf_counter() - t0
                    s1 = ctx.pipe_stats()
                    assert rc == 0 and not st.any()
                    row["calls"].append({"s": round(el, 4), "warm": rep == 0,
                                         **{key: s1[key] - s0[key] for key in ("sdma_checks", "sdma_slow",
                                                                              "sdma_down_checks", "sdma_down_slow",
                                                                              "verify_groups",
                                                                              "wave_blocks", "copies_1d",
                                                                              "copies_2d")},
                                         "sdma_last_mbps": s1["sdma_last_mbps"],
                                         "sdma_down_last_mbps": s1["sdma_down_last_mbps"]})
                timed = sorted(c["s"] for c in row["calls"][1:])
                row["median_s"] = timed[len(timed) // 2]
                ctx.close()
                print(json.dumps(row), flush=True)
        base.host_free(buf)
    base.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
