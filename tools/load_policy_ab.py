#!/usr/bin/env python3
"""Within-process A/B of RS kernel knobs on the bench's own buffers,
alternating rounds, HIP-event timed; then the guide's float4 copy on the
same buffers.  Config 2 and the north-star shape.  Lab tool, not product.

  python tools/load_policy_ab.py [--rounds 4] [--reps 10]
      nontemporal loads (default) vs plain loads, both with nontemporal
      stores (MXEC_RS_LOAD_NT, read per launch)
  python tools/load_policy_ab.py --env MXEC_RS_BPC --values 512,1024,2048
      any knob read per launch, one arm per value ("" = unset)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# The lab knobs exist only in the lab build (make -C maxio_amd/csrc lab).
os.environ.setdefault("MXEC_LIB", os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so"))

import bench  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="2,ns")
    ap.add_argument("--env", default="MXEC_RS_LOAD_NT")
    ap.add_argument("--values", default="1,0")
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
            for val in a.values.split(","):
                if val:
                    os.environ[a.env] = val
                else:
                    os.environ.pop(a.env, None)
                ms = bench.event_ms(torch, st, w.step, a.reps)
                print(json.dumps({"config": cfg, "round": rnd, a.env: val, "ms": round(ms, 4),
                                  "TBps": round(w.alg_bytes / (ms * 1e-3) / 1e12, 4)}), flush=True)
        os.environ.pop(a.env, None)
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
