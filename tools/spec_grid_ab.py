#!/usr/bin/env python3
"""A/B of the verified host GET's settings on bench.py's e2e_host leg
(128 x 4+2 x 10 MiB from page-locked memory, two erasures per object, right
after the device-resident configs[1] batch was freed), every timed call
listed: each setting in a fresh child process (--child), rounds interleaved.
The parent never touches the GPU.

  python tools/spec_grid_ab.py --settings "cap:;nocap:MXEC_SPEC_BLOCKS=0" --rounds 2 --reps 8 --lab
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(reps: int) -> None:
    sys.path.insert(0, ROOT)
    import torch

    import bench
    import maxio_amd

    plan = bench.plan_devices(1, os.environ, torch.cuda.device_count())
    ctx = maxio_amd.Context(streams_per_device=2)
    # the bench's state before its host legs: a large device batch, freed
    big = torch.empty(int(os.environ.get("SPEC_AB_HBM_GB", "60")) << 30, dtype=torch.uint8, device="cuda")
    big.fill_(1)
    torch.cuda.synchronize()
    del big
    torch.cuda.empty_cache()
    r = bench.e2e_host_leg(ctx, torch, plan, 128, reps=reps)
    out = {k: r[k]["s_each"] for k in ("rs_sha256", "get_verify_sha256")}
    out["get_counters"] = {k: r["get_verify_sha256"]["copies"][k] for k in ("spec_pieces", "wave_blocks", "copies_1d")}
    print(json.dumps(out), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default="default:")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--lab", action="store_true")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.reps)
        return 0
    for r in range(a.rounds):
        for spec in a.settings.split(";"):
            name, _, kv = spec.partition(":")
            env = dict(os.environ)
            env.update(dict(x.split("=", 1) for x in kv.split(",") if x))
            if a.lab:
                env["MXEC_LIB"] = os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so")
            out = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--reps", str(a.reps)],
                                 env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stderr[-3000:], file=sys.stderr)
                return out.returncode
            d = json.loads(out.stdout.strip().splitlines()[-1])
            g = sorted(d["get_verify_sha256"])
            print(json.dumps({"round": r, "setting": name, "get_median": g[len(g) // 2], "get_max": g[-1], **d}),
                  flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
