#!/usr/bin/env python3
"""HBM bytes per bench step of a workload whose step is several RS launches
(config 5's grouped / multi-r encode and reconstruct), from two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE) over `bench.py --config 5`: the sum
over every dispatch whose name holds `kernel`, divided by the steps the run
executed (the tuning launches before the warmup, warmup and timed), with the gfx950 correction of MI355X_MICROARCH.md
(read bytes = 2 x FETCH_SIZE KiB x 1024, write = WRITE_SIZE KiB x 1024).
The algorithmic bytes per step come from the run's own bench line
(roofline.bytes_per_launch).  The summary records blocks_per_cu, the grid of
the grouped launches (bench.py pmc_traffic matches it).

  python tools/pmc_step_summary.py fetch.csv write.csv bench_line.json --steps 4 --kernel rs_apply \\
      --blocks-per-cu 512 --tag cfg5_grouped --out profiles/r6_pmc_cfg5_grouped_traffic.json
"""
from __future__ import annotations

import argparse
import collections
import csv
import json


def total(path: str, counter: str, kernel: str):
    s, kinds = 0.0, collections.Counter()
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                s += float(r["Counter_Value"])
                kinds[r["Kernel_Name"].split("(")[0][:90]] += 1
    return s, kinds


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("line")
    ap.add_argument("--steps", type=int, default=0,
                    help="steps the run executed (default: the line's tuning launches + warmup + steps)")
    ap.add_argument("--kernel", default="rs_apply")
    ap.add_argument("--blocks-per-cu", type=int, required=True)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, kinds = total(a.fetch, "FETCH_SIZE", a.kernel)
    write, _ = total(a.write, "WRITE_SIZE", a.kernel)
    line = None
    for ln in open(a.line):
        if ln.startswith("{"):
            line = json.loads(ln)
    alg = float(line["roofline"]["bytes_per_launch"])
    if not a.steps:
        a.steps = int(line["tuning"]["launches"]) + int(line["warmup"]) + int(line["steps"])
    rd, wr = 2 * fetch * 1024 / a.steps, write * 1024 / a.steps
    out = {"kernel": a.kernel, "what": f"bench.py --config {line['config'].get('bench_config')}: every "
           f"{a.kernel} dispatch of {a.steps} steps (warmup + timed), per step; alg bytes = the line's "
           "roofline.bytes_per_launch (one step)", "dispatches": dict(kinds), "steps": a.steps,
           "correction": "gfx950: read bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024",
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (rd + wr) / alg,
           "blocks_per_cu": a.blocks_per_cu}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
