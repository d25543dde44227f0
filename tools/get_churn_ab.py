#!/usr/bin/env python3
"""The verified host GET (--objects x 4+2 x 10 MiB from page-locked memory, two
erasures per object; bench.py's _GetBatch) healthy and right after a large
HBM free: per setting a fresh child process (--child) that times `reps`
GETs back to back ("fresh"), then `reps` GETs each right after torch
allocates, fills and frees `--churn-gb` GB of HBM ("churn").  Rounds
interleaved; the parent never touches the GPU.

  python tools/get_churn_ab.py --settings "sdma:;waves:MXEC_SPEC_DOWN_WAVES=1" --lab
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(reps: int, churn_gb: int, objects: int) -> None:
    sys.path.insert(0, ROOT)
    import torch

    import bench
    import maxio_amd

    ctx = maxio_amd.Context(streams_per_device=2)
    shapes = [(4, 2, 10 << 20)] * objects
    rows, dig, _, _, _ = bench._encoded_set(ctx, shapes, 51)
    get = bench._GetBatch(ctx, shapes, rows, dig, 52)
    if os.environ.get("GET_RS_ONLY") == "1":  # the RS-only GET (no digests to verify)
        get.dig = None
    get.run()

    probes = []

    def timed():
        t0 = time.perf_counter()
        get.run()
        el = round(time.perf_counter() - t0, 4)
        st = ctx.pipe_stats()
        probes.append((st["sdma_down_checks"], st["sdma_down_slow"], st["sdma_down_last_mbps"]))
        return el

    fresh = [timed() for _ in range(reps)]
    churn = []
    for _ in range(reps if churn_gb > 0 else 0):
        big = torch.empty(churn_gb << 30, dtype=torch.uint8, device="cuda")
        big.fill_(1)
        torch.cuda.synchronize()
        del big
        torch.cuda.empty_cache()
        churn.append(timed())
    s = ctx.pipe_stats()
    print(json.dumps({"fresh": fresh, "churn": churn, "exact": bool(get.exact()),
                      "down_probes_checks_slow_mbps": probes,
                      "counters": {k: s[k] for k in ("spec_pieces", "wave_blocks", "copies_1d", "sdma_checks", "sdma_slow")}}), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default="default:")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--churn-gb", type=int, default=60)
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--lab", action="store_true")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.reps, a.churn_gb, a.objects)
        return 0
    for r in range(a.rounds):
        for spec in a.settings.split(";"):
            name, _, kv = spec.partition(":")
            env = dict(os.environ)
            env.update(dict(x.split("=", 1) for x in kv.split(",") if x))
            if a.lab:
                env["MXEC_LIB"] = os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so")
            out = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--reps", str(a.reps),
                                  "--churn-gb", str(a.churn_gb), "--objects", str(a.objects)], env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stderr[-3000:], file=sys.stderr)
                return out.returncode
            d = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps({"round": r, "setting": name, "fresh_median": statistics.median(d["fresh"]),
                              "churn_median": statistics.median(d["churn"]) if d["churn"] else None, **d}),
                  flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
