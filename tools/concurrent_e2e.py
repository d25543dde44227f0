"""Concurrent host-batch calls (bench.py e2e_concurrent) in fresh contexts
under different settings, one JSON line per setting: the PUT-with-digests +
verified-GET pair against its solo times, and the configs[4] mixed stream.

    python tools/concurrent_e2e.py --settings "lanes4:MXEC_PIPE_LANES=4;lanes1:MXEC_PIPE_LANES=1" \
        --objects 128 --reps 3 --seconds 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default="default:")
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=5.0)
    args = ap.parse_args()
    import torch  # noqa: F401  (the same HIP runtime as bench.py)

    import bench
    import maxio_amd

    for spec in args.settings.split(";"):
        name, _, env = spec.partition(":")
        kv = dict(x.split("=", 1) for x in env.split(",") if x)
        saved = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        try:
            ctx = maxio_amd.Context(streams_per_device=2)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        try:
            r = bench.e2e_concurrent(ctx, n=args.objects, reps=args.reps, stream_s=args.seconds)
        finally:
            ctx.close()
        print(json.dumps({"setting": name, "env": kv, **r}), flush=True)


if __name__ == "__main__":
    main()
