#!/usr/bin/env python3
"""Host <-> device copies by SDMA (hipMemcpyAsync) against copies by CU
waves reading / writing page-locked host memory directly
(libmaxio_probe mxprobe_copy_waves), HIP-event timed, median of --reps:

* whole-buffer rates, H2D and D2H, for several grid sizes;
* the pipeline's shape: --pieces copies of 1 MiB (hipMemcpyAsync each) vs one
  wave-copy launch per piece;
* both again right after freeing --churn-gib of torch buffers (the GET-stall
  study, DESIGN §7: after a large free the SDMA copies slow down for seconds).

Lab tool.  python tools/host_copy_lab.py [--gib 4] [--churn-gib 60]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grids", default="64,128,256,512,1024")
    ap.add_argument("--churn-gib", type=int, default=60)
    a = ap.parse_args()
    import torch

    import bench

    probe = bench.probe_lib()
    probe.mxprobe_copy_waves.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                         ctypes.c_void_p]
    probe.mxprobe_copy_waves.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    n = a.gib << 30
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    host.random_(0, 256)
    devb = torch.empty(n, dtype=torch.uint8, device=dev)
    hp, dp = host.data_ptr(), devb.data_ptr()

    def ms_of(fn, reps=a.reps):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        fn()
        torch.cuda.synchronize()
        out = []
        for e0, e1 in ev:
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1))
        return statistics.median(out), out

    def sdma(nbytes, kind):
        with torch.cuda.stream(st):
            if kind == "h2d":
                devb[:nbytes].copy_(host[:nbytes], non_blocking=True)
            else:
                host[:nbytes].copy_(devb[:nbytes], non_blocking=True)

    def pieces_sdma(kind, piece=1 << 20):
        with torch.cuda.stream(st):
            for o in range(0, n, piece):
                if kind == "h2d":
                    devb[o:o + piece].copy_(host[o:o + piece], non_blocking=True)
                else:
                    host[o:o + piece].copy_(devb[o:o + piece], non_blocking=True)

    def waves(kind, blocks, piece=0):
        step = piece or n
        for o in range(0, n, step):
            src, dst = (hp + o, dp + o) if kind == "h2d" else (dp + o, hp + o)
            rc = probe.mxprobe_copy_waves(dst, src, min(step, n - o), blocks, sh)
            assert rc == 0, rc

    def run(tag):
        row = {"phase": tag}
        for kind in ("h2d", "d2h"):
            ms, _ = ms_of(lambda: sdma(n, kind))
            row[f"sdma_{kind}_GBps"] = round(n / ms / 1e6, 1)
            ms, each = ms_of(lambda: pieces_sdma(kind))
            row[f"sdma_{kind}_1MiB_pieces_GBps"] = round(n / ms / 1e6, 1)
            row[f"sdma_{kind}_1MiB_pieces_ms_each"] = [round(x, 1) for x in each]
            for g in a.grids.split(","):
                ms, _ = ms_of(lambda: waves(kind, int(g)))
                row[f"waves{g}_{kind}_GBps"] = round(n / ms / 1e6, 1)
            ms, _ = ms_of(lambda: waves(kind, 256, 1 << 20))
            row[f"waves256_{kind}_1MiB_launches_GBps"] = round(n / ms / 1e6, 1)
        ok = torch.equal(devb[:1 << 20].cpu(), host[:1 << 20])
        row["bytes_equal"] = bool(ok)
        print(json.dumps(row), flush=True)

    run("fresh")
    if a.churn_gib:
        t = torch.empty(a.churn_gib << 30, dtype=torch.uint8, device=dev)
        t.fill_(1)
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        run(f"right after freeing {a.churn_gib} GiB")
        print(json.dumps({"churn_phase_s": round(time.perf_counter() - t0, 2)}), flush=True)
        time.sleep(10)
        run("10 s later")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
