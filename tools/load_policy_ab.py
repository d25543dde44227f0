#!/usr/bin/env python3
"""Within-process A/B of the RS kernel's load form on the bench's own
buffers: nontemporal loads (default) vs plain loads, both with nontemporal
stores (MXEC_RS_LOAD_NT, read per launch), alternating rounds, HIP-event
timed; then the guide's float4 copy on the same buffers.  Config 2 and the
north-star shape.  Lab tool, not product.

  python tools/load_policy_ab.py [--rounds 4] [--reps 10]
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
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="2,ns")
    a = ap.parse_args()
    import torch

    import maxio_amd

    dev = torch.device("cuda", 0)
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    st = torch.cuda.Stream(device=dev)
    for cfg in a.configs.split(","):
        w = bench.make_workload(cfg, torch, ctx, dev, st.cuda_stream, 0, 0)
        torch.cuda.synchronize()
        for rnd in range(a.rounds):
            for mode in ("1", "0"):
                os.environ["MXEC_RS_LOAD_NT"] = mode
                ms = bench.event_ms(torch, st, w.step, a.reps)
                print(json.dumps({"config": cfg, "round": rnd, "load_nt": mode == "1", "ms": round(ms, 4),
                                  "TBps": round(w.alg_bytes / (ms * 1e-3) / 1e12, 4)}), flush=True)
        os.environ["MXEC_RS_LOAD_NT"] = "1"
        ok = w.spot_check()
        f4 = bench.float4_copy_on_buffers(torch, st, w)
        print(json.dumps({"config": cfg, "spot_check": ok, "float4_copy_same_buffers_GBps": f4}), flush=True)
        w.drop()
        del w
        torch.cuda.empty_cache()
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
