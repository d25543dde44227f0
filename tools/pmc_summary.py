#!/usr/bin/env python3
"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), with the gfx950 correction of MI355X_MICROARCH.md:
FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so read
bytes = 2 x FETCH_SIZE KiB x 1024; WRITE_SIZE is exact.

  python tools/pmc_summary.py <fetch_dir|csv> <write_dir|csv> <kernel-substring> <alg_bytes_per_launch>
      [--blocks-per-cu N --cus 256] [--out f.json]

--blocks-per-cu records the grid the kernel ran at (bench.py's pmc_traffic
only uses a summary whose blocks_per_cu equals the timed kernel's); when the
CSV carries Grid_Size, the measured grid must equal min(--tiles, bpc x cus)
workgroups.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os


def per_launch(d: str, counter: str, kernel: str, grids=None) -> tuple[float, int]:
    vals = []
    paths = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "*counter_collection.csv"))
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                    vals.append(float(r["Counter_Value"]))
                    if grids is not None and r.get("Grid_Size"):
                        grids.add(int(float(r["Grid_Size"])))
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
    ap.add_argument("--blocks-per-cu", type=int, default=None)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--threads", type=int, default=256, help="work-items per workgroup")
    ap.add_argument("--tiles", type=int, default=None, help="tiles per launch (the grid is min(tiles, bpc x cus))")
    a = ap.parse_args()
    grids: set = set()
    fk, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel, grids)
    wk, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel, grids)
    if a.blocks_per_cu and grids:
        blocks = a.blocks_per_cu * a.cus
        if a.tiles:
            blocks = min(blocks, a.tiles)
        want = blocks * a.threads
        if grids != {want}:
            raise SystemExit(f"Grid_Size {sorted(grids)} != {blocks} workgroups x {a.threads}: "
                             "the profiled launches ran at another grid")
    rd, wr = 2 * fk * 1024, wk * 1024
    out = {
        "kernel": a.kernel, "what": a.what,
        "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk, "launches": [nf, nw],
        "correction": "gfx950: read bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024",
        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": a.alg_bytes,
        "traffic_over_algorithmic": (rd + wr) / a.alg_bytes,
    }
    if a.blocks_per_cu:
        out["blocks_per_cu"] = a.blocks_per_cu
        out["grid_size_measured"] = sorted(grids) or None
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
