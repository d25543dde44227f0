#!/usr/bin/env python3
"""Two questions about HIP streams on this box, each in a fresh child
process (the queue a new stream lands on depends on what the process
created before):

* do two streams created with complementary CU masks (even / odd CUs) run
  a busy-wait kernel each at the same time (their own queues, or one shared)?
* do two small launches on two plain streams land on the same CUs?  A
  one-workgroup busy kernel per stream, timed alone and side by side.

  python tools/queue_probe2.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

CHILD = r'''
import ctypes, glob, json, os, sys, time
import torch
torch.cuda.set_device(0)
torch.cuda._sleep(1000); torch.cuda.synchronize()
hip = None
for lib in sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))) + ["libamdhip64.so"]:
    try:
        hip = ctypes.CDLL(lib); break
    except OSError:
        pass
n_cus = torch.cuda.get_device_properties(0).multi_processor_count
words = (n_cus + 31) // 32
def masked(parity):
    m = [0] * words
    for c in range(n_cus):
        if c % 2 == parity:
            m[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint32 * words)(*m)
    h = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), arr) == 0
    return torch.cuda.ExternalStream(h.value)
def run(ss, cyc=40_000_000):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(cyc)
    torch.cuda.synchronize(); return time.perf_counter() - t0
mode = sys.argv[1]
if mode == "masked":
    ss = [masked(0), masked(1)]
elif mode == "masked_after4":
    keep = [torch.cuda.Stream() for _ in range(4)]
    ss = [masked(0), masked(1)]
else:
    ss = [torch.cuda.Stream(), torch.cuda.Stream()]
run(ss[:1]); one = run(ss[:1]); run(ss); two = run(ss)
print(json.dumps({"mode": mode, "one_s": round(one, 4), "two_side_by_side_s": round(two, 4), "ratio": round(two / one, 2)}))
'''


def main() -> int:
    for mode in ("plain", "masked", "masked_after4"):
        out = subprocess.run([sys.executable, "-c", CHILD, mode], capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:], file=sys.stderr)
            return out.returncode
        print(out.stdout.strip().splitlines()[-1], flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
