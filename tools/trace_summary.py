#!/usr/bin/env python3
"""Per-shape kernel durations from a rocprofv3 kernel trace.

rocprofv3's --stats summary averages every launch of a kernel symbol, and the
default `bench.py` run launches rs_apply_fast<2,4,true> for the headline
encode (1024 x 4+2 x 10 MiB, 11-12 ms) and for the extras' decodes (2-9 ms),
so its average is not the headline launch's.  This groups the trace's
launches by (kernel, grid, workgroup) and prints count / average / min / max
per group, the figure to set beside the bench line's HIP-event
ms_per_launch.

  python tools/trace_summary.py <kernel_trace.csv> [--match rs_apply_fast] [--out f.json]
  python tools/trace_summary.py <trace> --match 'rs_apply_fast<2' --skip 3 --first 20
      launches 4..23 of the match in start order (bench.py's timed steps
      after --warmup 3), as one group
"""
from __future__ import annotations

import argparse
import collections
import csv
import json


def summarize(path: str, match: str, skip: int = 0, first: int = 0) -> list[dict]:
    groups = collections.defaultdict(list)
    order = []
    with open(path) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if not match or match in r["Kernel_Name"]]
    if first:
        rows = rows[skip: skip + first]
    for r in rows:
        key = (r["Kernel_Name"], int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0),
               int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0))
        if key not in groups:
            order.append(key)
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = []
    for key in order:
        ms = groups[key]
        out.append({"kernel": key[0][:160], "grid": key[1], "workgroup": key[2], "launches": len(ms),
                    "avg_ms": round(sum(ms) / len(ms), 4), "min_ms": round(min(ms), 4),
                    "max_ms": round(max(ms), 4)})
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip", type=int, default=0, help="with --first: launches of the match to skip")
    ap.add_argument("--first", type=int, default=0, help="only this many launches of the match, in start order")
    a = ap.parse_args()
    rows = summarize(a.trace, a.match, a.skip, a.first)
    for r in rows:
        print(json.dumps(r))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"source": "rocprofv3 --kernel-trace, launches grouped by (kernel, grid, workgroup)",
                       "groups": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
