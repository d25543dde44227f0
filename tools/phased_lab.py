#!/usr/bin/env python3
"""Does time-dividing the RS pattern into read and write phases beat the
steady 2:1 mix?  The RS pattern's reads alone and writes alone each run
~6.8 TB/s where both together run ~6.0 (box 8); here every
workgroup reads G tiles (parity in registers) only in the first `rwin` ticks
of each `period` of the chip-wide 100 MHz clock and stores only in the rest
(libmaxio_probe mxprobe_rs_phased).  One configs[1]-shaped object-major batch
(4+2 x 10 MiB, pad 2 MiB + 64 KiB), HIP-event timed, median of --reps; one
JSON line per setting, plus the ungated kernel, the usual pattern probe and
the float4 copy on the same buffer.  Lab tool.

  python tools/phased_lab.py [--objects 512] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--periods", default="1000,2000,4000,8000", help="ticks of 10 ns")
    ap.add_argument("--fracs", default="0.6,0.67,0.75", help="read share of each period")
    a = ap.parse_args()
    import torch

    import bench

    k, m, S, n = 4, 2, 10 << 20, a.objects
    ss = S + (2 << 20) + (64 << 10)
    ost = (k + m) * ss
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    probe = bench.probe_lib()
    probe.mxprobe_rs_phased.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    probe.mxprobe_rs_phased.restype = ctypes.c_int
    obj = torch.empty((n, k + m, ss), dtype=torch.uint8, device=dev)
    obj[:, :k, :S].random_(0, 256)
    torch.cuda.synchronize()
    d0, p0 = obj.data_ptr(), obj[:, k:].data_ptr()
    alg = n * (k + m) * S

    def tbps(ms):
        return round(alg / (ms * 1e-3) / 1e12, 4)

    def phased(G, wpc, period, rwin):
        def f():
            rc = probe.mxprobe_rs_phased(d0, p0, S, n, ost, ss, G, wpc, period, rwin, sh)
            assert rc == 0, rc
        return tbps(bench.event_ms(torch, st, f, a.reps, warm=1))

    base = {"objects": n,
            "pattern_TBps": tbps(bench.event_ms(torch, st, lambda: probe.mxprobe_rs_pattern_strided(
                d0, p0, k, m, S, n, ost, ost, ss, sh), a.reps))}
    half = (obj.numel() // 2) & ~15
    ms = bench.event_ms(torch, st, lambda: probe.mxprobe_copy_float4(d0 + half, d0, half, sh), a.reps)
    base["f4copy_TBps"] = round(2 * half / (ms * 1e-3) / 1e12, 4)
    for G, wpcs in ((1, (4, 8, 16)), (2, (2, 4, 8)), (4, (1, 2, 4))):
        for wpc in wpcs:
            base[f"ungated_G{G}_wpc{wpc}_TBps"] = phased(G, wpc, 0, 0)
    print(json.dumps(base), flush=True)
    for G, wpc in ((1, 8), (2, 4), (4, 2)):
        for period in (int(x) for x in a.periods.split(",")):
            row = {"G": G, "wpc": wpc, "period_ticks": period}
            for fr in (float(x) for x in a.fracs.split(",")):
                row[f"r{fr}_TBps"] = phased(G, wpc, period, int(period * fr))
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
