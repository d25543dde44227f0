#!/usr/bin/env python3
"""mxec_batch_alloc over a configs[1] batch (1024 x 4+2 x 10 MiB) several
times in one process, torch holding a different amount of HBM before each
call so the allocations land in different places: the probed layouts'
encode times (allocation-major, two strides each) and the stride kept, one
JSON line per call.  Shows whether "slow" placements (~11.1 ms against
~10.3) turn up among the candidates and are passed over.

  python tools/placement_probe.py --calls 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=6)
    ap.add_argument("--spacer-gb", default="0,3,7,13,21,1")
    a = ap.parse_args()
    import torch

    import maxio_amd

    ctx = maxio_amd.Context(streams_per_device=2)
    k, m, S, n = 4, 2, 10 << 20, 1024
    spacers = [int(x) for x in a.spacer_gb.split(",")]
    for i in range(a.calls):
        gb = spacers[i % len(spacers)]
        spacer = torch.empty(gb << 30, dtype=torch.uint8, device="cuda") if gb else None
        p, stride, probe = ctx.batch_alloc(k, m, S, n)
        ctx.batch_free(p)
        del spacer
        torch.cuda.synchronize()
        probe = [round(x, 3) for x in probe]
        kept = min(x for x in probe if x > 0)
        print(json.dumps({"call": i, "spacer_GB": gb, "probe_ms": probe, "kept_ms": kept, "stride": stride,
                          "slowest_ms": max(probe), "slow_candidates": sum(1 for x in probe if x > 10.9)}),
              flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
