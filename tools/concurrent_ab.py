#!/usr/bin/env python3
"""A/B of host-pipeline settings on concurrent host batches (bench.py
e2e_concurrent: the PUT-with-digests + verified-GET pair against its solo
times, and optionally the configs[4] mixed stream), each setting in a fresh
child process, rounds interleaved so box drift hits every setting alike.
The parent never touches the GPU.

  python tools/concurrent_ab.py --settings "spec:;nospec:MXEC_GET_SPECULATE=0" --rounds 3 --seconds 0
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default="default:")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=0.0)
    ap.add_argument("--lab", action="store_true", help="load the lab build (MXEC_LIB) in the children")
    a = ap.parse_args()
    env0 = dict(os.environ)
    if a.lab:
        env0["MXEC_LIB"] = os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so")
    for r in range(a.rounds):
        for spec in a.settings.split(";"):
            out = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "concurrent_e2e.py"),
                                  "--settings", spec, "--objects", str(a.objects), "--reps", str(a.reps),
                                  "--seconds", str(a.seconds)], env=env0, capture_output=True, text=True,
                                 timeout=600)
            if out.returncode != 0:
                print(out.stderr[-3000:], file=sys.stderr)
                return out.returncode
            for line in out.stdout.strip().splitlines():
                d = json.loads(line)
                p = d["pair"]
                print(json.dumps({"round": r, "setting": d["setting"], "solo_put_s": p["solo_put_s"],
                                  "solo_get_s": p["solo_get_s"], "pair_s": p["pair_s"],
                                  "pair_over_solo_sum": p["pair_over_solo_sum"], "finish": p["finish_times_s"],
                                  "counters": p["counters"], "spot_check": p["spot_check"],
                                  **({"mixed_stream": d["mixed_stream"]} if "mixed_stream" in d else {})}),
                      flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
