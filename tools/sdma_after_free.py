#!/usr/bin/env python3
"""SDMA copy rates right after a large HBM free (the GET-slowdown study).

Host batch GETs by SDMA ran 20-30 % slower (and PUT with digests at 512
objects 2.4x slower) in the seconds after tens of GB of HBM were freed,
while CU-wave copies did not (tools/watch_diag.py --churn-each).
This times plain page-locked <-> HBM copies (hipMemcpyAsync through torch,
HIP events) before and after one free, one direction at a time and both at
once, to see which direction slows, by how much and for how long.

  python tools/sdma_after_free.py [--free-gb 60] [--seconds 8] [--mib 512]

One JSON line per sample: {"t": s since the free (negative: before), "dir":
"d2h" | "h2d" | "duplex_d2h" | "duplex_h2d", "GBps": ...}; then a summary.
"""
from __future__ import annotations

import argparse
import json
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--free-gb", type=float, default=60.0)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--mib", type=int, default=512)
    a = ap.parse_args()
    import torch

    n = a.mib << 20
    host_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    host_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
    host_src.fill_(3)
    dev_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev_a.fill_(5)
    s_up, s_dn = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(direction: str) -> list[tuple[str, float]]:
        out = []
        pairs = []
        if direction in ("h2d", "duplex"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s_up):
                e0.record()
                dev_b.copy_(host_src, non_blocking=True)
                e1.record()
            pairs.append(("duplex_h2d" if direction == "duplex" else "h2d", e0, e1, s_up))
        if direction in ("d2h", "duplex"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s_dn):
                e0.record()
                host_dst.copy_(dev_a, non_blocking=True)
                e1.record()
            pairs.append(("duplex_d2h" if direction == "duplex" else "d2h", e0, e1, s_dn))
        for name, e0, e1, s in pairs:
            s.synchronize()
            out.append((name, n / (e0.elapsed_time(e1) * 1e6)))
        return out

    rows = []
    t_free = None

    def sample(t: float) -> None:
        for d in ("d2h", "h2d", "duplex"):
            for name, gbps in timed(d):
                r = {"t": round(t, 3), "dir": name, "GBps": round(gbps, 2)}
                rows.append(r)
                print(json.dumps(r), flush=True)

    for _ in range(3):  # before
        sample(-1.0)
    big = torch.empty(int(a.free_gb * 1e9), dtype=torch.uint8, device="cuda")
    big.fill_(1)
    torch.cuda.synchronize()
    del big
    t0 = time.perf_counter()
    torch.cuda.empty_cache()
    t_free = time.perf_counter() - t0
    while time.perf_counter() - t0 < a.seconds:
        sample(time.perf_counter() - t0)
    summ = {"free_gb": a.free_gb, "empty_cache_s": round(t_free, 4), "copy_MiB": a.mib}
    for d in ("d2h", "h2d", "duplex_d2h", "duplex_h2d"):
        before = [r["GBps"] for r in rows if r["dir"] == d and r["t"] < 0]
        after = [(r["t"], r["GBps"]) for r in rows if r["dir"] == d and r["t"] >= 0]
        base = sorted(before)[len(before) // 2]
        slow = [t for t, g in after if g < 0.85 * base]
        summ[d] = {"before_GBps": base, "after_min_GBps": min(g for _, g in after),
                   "slow_until_s": round(max(slow), 3) if slow else 0.0,
                   "after_first3": [g for _, g in after[:3]]}
    print(json.dumps({"summary": summ}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
