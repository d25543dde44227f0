#!/usr/bin/env python3
"""Do kernels on different HIP streams overlap?  GPU_MAX_HW_QUEUES (4 here)
hardware queues per process serve every stream; streams beyond that share a
queue, and kernels of streams that share one run in submission order.  One
busy-wait kernel (torch.cuda._sleep, ~20 ms) per stream on N fresh streams
at once: wall time / one kernel's time = how many ran one after another.
Also with the streams at the highest priority (their own queue pool).

  python tools/queue_probe.py --streams 2,4,6,8
"""
from __future__ import annotations

import argparse
import json
import os
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4,5,6,8")
    ap.add_argument("--cycles", type=int, default=40_000_000)
    a = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)

    def one(streams):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(a.cycles)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    base = one([torch.cuda.Stream()])
    # Streams with a CU mask (every CU set) from hipExtStreamCreateWithCUMask
    # beside four plain ones: do they get queues of their own?
    import ctypes
    import glob
    hip = None
    for lib in sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))) + ["libamdhip64.so"]:
        try:
            hip = ctypes.CDLL(lib)
            break
        except OSError:
            continue
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n_cus + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))

    def masked():
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
        assert rc == 0, rc
        return torch.cuda.ExternalStream(h.value)

    plain4 = [torch.cuda.Stream() for _ in range(4)]
    for n in (1, 2, 4):
        ms = [masked() for _ in range(n)]
        one(plain4 + ms)
        el = one(plain4 + ms)
        print(json.dumps({"streams": f"4 plain + {n} CU-masked (all CUs)", "s": round(el, 4),
                          "one_kernel_s": round(base, 4), "serialised_x": round(el / base, 2)}), flush=True)
    for n in [int(x) for x in a.streams.split(",")]:
        for prio in ("normal", "high", "mixed"):
            if prio == "normal":
                ss = [torch.cuda.Stream() for _ in range(n)]
            elif prio == "high":
                ss = [torch.cuda.Stream(priority=hi) for _ in range(n)]
            else:
                ss = [torch.cuda.Stream(priority=hi if i % 2 else 0) for i in range(n)]
            one(ss)
            el = one(ss)
            print(json.dumps({"streams": n, "priority": prio, "s": round(el, 4), "one_kernel_s": round(base, 4),
                              "serialised_x": round(el / base, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
