#!/usr/bin/env python3
"""The bench's end-to-end host leg (bench.e2e_host_leg) several times in one
process, every batch's time printed: where its outliers come from.  Lab
tool, not product.

  python tools/e2e_reps.py [--runs 3] [--objects 128]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--objects", type=int, default=128)
    a = ap.parse_args()
    import torch

    import maxio_amd

    plan = bench.plan_devices(1, os.environ, torch.cuda.device_count())
    ctx = maxio_amd.Context(device_mask=plan.device_mask, streams_per_device=2)
    for r in range(a.runs):
        res = bench.e2e_host_leg(ctx, torch, plan, a.objects)
        print(json.dumps({"run": r, "MXEC_HOST_NUMA": os.environ.get("MXEC_HOST_NUMA"), "numa": res.get("numa"),
                          **{k: res[k]["s_each"] for k in
                             ("rs_only", "rs_sha256", "get_rs_only", "get_verify_sha256")}}), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
