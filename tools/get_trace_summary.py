#!/usr/bin/env python3
"""Where a verified GET batch's wall time goes, from a rocprofv3 kernel +
memory-copy trace of bench.py run with BENCH_GET_STAMPS=1 (each timed GET
batch's CLOCK_MONOTONIC start / end in the bench line).  Lab tool.

Per batch: wall time, busy time of kernels and copies (union of intervals),
per-kernel and per-direction totals, and the longest gaps with nothing on
the GPU and what ran either side of them.

  python tools/get_trace_summary.py kernel_trace.csv memory_copy_trace.csv bench.json [--out x.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import re


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def load(kt, mt):
    ev = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            name = _col(r, "Kernel_Name", "KernelName")
            short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)", ""))[:90]
            ev.append((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp")), "K", short, 0))
    with open(mt) as f:
        for r in csv.DictReader(f):
            d = _col(r, "Direction", "Kind")
            b = int(r.get("Bytes") or r.get("Size") or 0)
            ev.append((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp")), "C", d, b))
    ev.sort()
    return ev


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def gaps(ev, t0, t1, top=4):
    """Longest stretches of [t0, t1) with no kernel or copy running."""
    iv = sorted((max(s, t0), min(e, t1), kind, name) for (s, e, kind, name, _) in ev if e > t0 and s < t1)
    out, cur, prev = [], t0, "(batch start)"
    for s, e, kind, name in iv:
        if s > cur:
            out.append((s - cur, cur, prev, f"{kind}:{name}"))
        if e > cur:
            cur, prev = e, f"{kind}:{name}"
    if t1 > cur:
        out.append((t1 - cur, cur, prev, "(batch end)"))
    out.sort(reverse=True)
    return [{"gap_ms": round(g / 1e6, 3), "at_ms": round((c - t0) / 1e6, 3), "after": a, "before": b}
            for g, c, a, b in out[:top]]


def summarize(ev, t0, t1):
    inside = [x for x in ev if x[1] > t0 and x[0] < t1]
    per = {}
    for s, e, kind, name, b in inside:
        k = f"{kind}:{name}"
        d = per.setdefault(k, {"n": 0, "ms": 0.0, "bytes": 0})
        d["n"] += 1
        d["ms"] += (min(e, t1) - max(s, t0)) / 1e6
        d["bytes"] += b
    for d in per.values():
        d["ms"] = round(d["ms"], 3)
    return {"wall_ms": round((t1 - t0) / 1e6, 3),
            "busy_any_ms": round(union([(max(s, t0), min(e, t1)) for s, e, *_ in inside]) / 1e6, 3),
            "busy_kernels_ms": round(union([(max(s, t0), min(e, t1)) for s, e, k, *_ in inside if k == "K"]) / 1e6, 3),
            "busy_copies_ms": round(union([(max(s, t0), min(e, t1)) for s, e, k, *_ in inside if k == "C"]) / 1e6, 3),
            "by_item": dict(sorted(per.items(), key=lambda kv: -kv[1]["ms"])[:12]),
            "longest_idle_gaps": gaps(ev, t0, t1)}


def find_marks(obj, path=""):
    """(leg path, [(start, end)]) for every monotonic_ns list in the bench line."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k == "monotonic_ns":
                out.append((path, v))
            else:
                out += find_marks(v, f"{path}.{k}" if path else k)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel_trace")
    ap.add_argument("copy_trace")
    ap.add_argument("bench_json")
    ap.add_argument("--out")
    a = ap.parse_args()
    ev = load(a.kernel_trace, a.copy_trace)
    with open(a.bench_json) as f:
        line = json.loads([ln for ln in f if ln.strip().startswith("{")][-1])
    lo, hi = ev[0][0], max(e for _, e, *_ in ev)
    res = {"trace_span_ns": [lo, hi], "legs": {}}
    for path, marks in find_marks(line):
        res["legs"][path] = [dict(summarize(ev, s, e), batch=i, in_trace=bool(lo <= s <= hi))
                             for i, (s, e) in enumerate(marks)]
    text = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
