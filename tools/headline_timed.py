#!/usr/bin/env python3
"""The headline encode's launches in a rocprofv3 kernel trace of bench.py,
split into the phases the bench line reports: mxec_batch_alloc's placement
probes (three encodes per probed layout, `config.placement.probe_ms`), the
tuning launches
(`tuning.launches`, run before --warmup until the RS grid tuner decided),
the --warmup launches and the timed --steps launches.  Prints one JSON
object: the grids of each phase, whether every timed launch ran one grid,
and the timed launches' average / min / max duration next to the line's
HIP-event ms_per_launch (the two must agree).

  python tools/headline_timed.py <kernel_trace.csv> <bench.json> [--out f.json]
"""
from __future__ import annotations

import argparse
import csv
import json


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_json")
    ap.add_argument("--match", default="rs_apply_fast<2")
    ap.add_argument("--out", default=None)
    ap.add_argument("--min-frac", type=float, default=0.5,
                    help="launches shorter than this fraction of the line's ms_per_launch are not the headline's "
                         "(the host legs, which run before it, launch the same kernel over pieces of a batch)")
    a = ap.parse_args()
    line = None
    with open(a.bench_json) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    if line is None:
        raise SystemExit("no bench line in " + a.bench_json)
    tune = int(line.get("tuning", {}).get("launches", 0))
    probes = 3 * sum(1 for x in (line.get("config", {}).get("placement") or {}).get("probe_ms", []) if x > 0)
    warm, steps = int(line["warmup"]), int(line["steps"])
    def grid(r):
        return int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)

    def dur_ms(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6

    floor_ms = a.min_frac * float(line["roofline"]["ms_per_launch"])
    with open(a.trace) as f:
        rows = sorted((r for r in csv.DictReader(f) if a.match in r["Kernel_Name"] and dur_ms(r) >= floor_ms),
                      key=lambda r: int(r["Start_Timestamp"]))
    probe_rows, rows = rows[:probes], rows[probes: probes + tune + warm + steps]

    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[tune + warm:]]
    timed_grids = sorted({grid(r) for r in rows[tune + warm:]})
    out = {
        "source": f"{a.trace} (rocprofv3 --kernel-trace of bench.py) and {a.bench_json}",
        "command_steps_warmup": [steps, warm],
        "what": (f"the headline kernel ({a.match}..., launches of >= {floor_ms:.2f} ms: whole-batch encodes) in "
                 f"trace order: "
                 f"{probes} placement probe launches, "
                 f"{tune} tuning launches before the warmup (the grid tuner's trials), {warm} warmup, then the "
                 f"{steps} timed steps"),
        "placement_probe_grids": sorted({grid(r) for r in probe_rows}),
        "tuning_grids": [grid(r) for r in rows[:tune]],
        "warmup_grids": [grid(r) for r in rows[tune:tune + warm]],
        "timed_grids": timed_grids,
        "one_grid_over_timed_launches": len(timed_grids) == 1,
        "timed_launches": len(ms),
        "avg_ms": round(sum(ms) / len(ms), 4) if ms else None,
        "min_ms": round(min(ms), 4) if ms else None,
        "max_ms": round(max(ms), 4) if ms else None,
        "hip_event_ms_per_launch_same_run": line["roofline"]["ms_per_launch"],
        "tuner_decided_before_timing": line.get("tuner_decided_before_timing"),
        "blocks_per_cu": line["roofline"].get("blocks_per_cu"),
    }
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
