#!/usr/bin/env python3
"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), with the gfx950 correction of MI355X_MICROARCH.md:
FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so read
bytes = 2 x FETCH_SIZE KiB x 1024; WRITE_SIZE is exact.

  python tools/pmc_summary.py <fetch_dir|csv> <write_dir|csv> <kernel-substring> <alg_bytes_per_launch> [--out f.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def per_launch(d: str, counter: str, kernel: str) -> tuple[float, int]:
    vals = []
    paths = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "*counter_collection.csv"))
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                    vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel!r} under {d}")
    return sum(vals) / len(vals), len(vals)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("kernel")
    ap.add_argument("alg_bytes", type=float)
    ap.add_argument("--what", default="")
    ap.add_argument("--out")
    a = ap.parse_args()
    fk, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wk, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel)
    rd, wr = 2 * fk * 1024, wk * 1024
    out = {
        "kernel": a.kernel, "what": a.what,
        "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk, "launches": [nf, nw],
        "correction": "gfx950: read bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024",
        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": a.alg_bytes,
        "traffic_over_algorithmic": (rd + wr) / a.alg_bytes,
    }
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
