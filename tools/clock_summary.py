#!/usr/bin/env python3
"""Effective shader clock of each profiled kernel from a rocprofv3 --pmc pass
of GRBM_GUI_ACTIVE (and GRBM_COUNT), per MI355X_MICROARCH.md 'DVFS give-back':
clock = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) / dispatch wall time,
within ~3 % of the in-kernel clock for dispatches of 10 ms or more.

  python tools/clock_summary.py <csv|dir> [--kernel SUBSTR ...] [--what TEXT] [--out f.json]

Used for the latency-bound SHA-256 rooflines: a lone message's block costs
its consumer wave's instruction count x 4 cycles at the clock the chip holds,
not at the 2.4 GHz maximum (bench.py config 3 'chain' block).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics


def short(name: str) -> str:
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def rows(path: str):
    paths = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                           recursive=True)
    for p in paths:
        with open(p) as f:
            yield from csv.DictReader(f)


def summarize(path: str, kernels=None) -> dict:
    per: dict = {}
    for r in rows(path):
        k = short(r["Kernel_Name"])
        if kernels and not any(s in r["Kernel_Name"] for s in kernels):
            continue
        d = per.setdefault(k, {}).setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, disp in per.items():
        ok = [d for d in disp.values() if "GRBM_GUI_ACTIVE" in d and d["ns"] > 0]
        if not ok:
            continue
        clk = [d["GRBM_GUI_ACTIVE"] / 8 / d["ns"] for d in ok]
        ms = [d["ns"] / 1e6 for d in ok]
        e = {"dispatches": len(ok), "ms_median": round(statistics.median(ms), 4),
             "clock_GHz_median": round(statistics.median(clk), 4),
             "clock_GHz_min": round(min(clk), 4), "clock_GHz_max": round(max(clk), 4)}
        long_ = [c for c, t in zip(clk, ms) if t >= 10.0]
        if long_:
            e["clock_GHz_median_dispatches_ge_10ms"] = round(statistics.median(long_), 4)
        if all("GRBM_COUNT" in d for d in ok):
            e["GRBM_COUNT_over_8_per_ns_median"] = round(statistics.median(d["GRBM_COUNT"] / 8 / d["ns"] for d in ok), 4)
        out[k] = e
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", action="append", default=[])
    ap.add_argument("--what", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = summarize(a.path, a.kernel)
    if not res:
        raise SystemExit(f"no GRBM_GUI_ACTIVE rows under {a.path}")
    doc = {"what": a.what,
           "method": "clock = GRBM_GUI_ACTIVE / 8 / (End_Timestamp - Start_Timestamp), per dispatch "
                     "(MI355X_MICROARCH.md 'DVFS give-back'); dispatches serialised by counter collection",
           "kernels": res}
    s = json.dumps(doc, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
