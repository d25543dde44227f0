#!/usr/bin/env python3
"""GPU busy time of a window in a rocprofv3 kernel trace.

Finds the launches of `--match` (e.g. the kernels of bench.py's timed steps),
takes the window from the first of the last `--last` launches' start to the
trace's last end, and reports the window, the union of all kernel intervals
inside it (any stream) and the gaps: how much of a multi-stream step the chip
actually had a kernel resident.

  python tools/trace_busy.py <kernel_trace.csv> --match rs_apply --last 300
"""
from __future__ import annotations

import argparse
import csv
import json


def busy(path: str, match: str, last: int) -> dict:
    with open(path) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    hits = [i for i, r in enumerate(rows) if match in r["Kernel_Name"]]
    if not hits:
        return {"error": "no launch matches"}
    first = hits[-last] if last and len(hits) >= last else hits[0]
    t0 = iv[first][0]
    t1 = max(e for s, e in iv[first:])
    union, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv[first:]:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    gaps.sort()
    return {"window_ms": round((t1 - t0) / 1e6, 3), "busy_ms": round(union / 1e6, 3),
            "busy_frac": round(union / (t1 - t0), 4), "launches": len(iv) - first,
            "gaps": len(gaps), "gap_ms_total": round(sum(gaps) / 1e6, 3),
            "gap_us_p50": round(gaps[len(gaps) // 2] / 1e3, 1) if gaps else 0,
            "gap_us_max": round(gaps[-1] / 1e3, 1) if gaps else 0}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--last", type=int, default=0, help="window starts at the last N matching launches")
    a = ap.parse_args()
    print(json.dumps(busy(a.trace, a.match, a.last)))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
