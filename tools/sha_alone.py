#!/usr/bin/env python3
"""SHA-256 of n device-resident messages alone (mxec_sha256_batch_device),
HIP-event timed on its stream: the configs[2] hash launch without the
verify / rebuild around it, for A/B of library builds (MXEC_LIB), including
diagnostic builds whose digests are wrong (make nosched / nosync).

  python tools/sha_alone.py [--n 10240] [--mib 1] [--reps 5]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10240)
    ap.add_argument("--mib", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import maxio_amd

    torch.cuda.set_device(0)
    S = a.mib << 20
    buf = torch.randint(0, 256, (a.n, S), dtype=torch.uint8, device="cuda")
    dig = torch.zeros((a.n, 32), dtype=torch.uint8, device="cuda")
    ptrs = [buf[i].data_ptr() for i in range(a.n)]
    lens = [S] * a.n
    s = torch.cuda.Stream()
    with maxio_amd.Context(device_mask=1, streams_per_device=2) as ctx:
        ctx.sha256_batch_device(ptrs, lens, dig.data_ptr(), stream=s.cuda_stream)  # warm
        s.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ctx.sha256_batch_device(ptrs, lens, dig.data_ptr(), stream=s.cuda_stream)
            e1.record(s)
            s.synchronize()
            ms.append(e0.elapsed_time(e1))
        ok = bytes(dig[a.n // 2].cpu().numpy()) == hashlib.sha256(buf[a.n // 2].cpu().numpy().tobytes()).digest()
    ms.sort()
    med = ms[len(ms) // 2]
    print(json.dumps({"lib": os.path.basename(os.environ.get("MXEC_LIB", "libmaxio_ec.so")), "n": a.n, "MiB": a.mib,
                      "ms": round(med, 3), "ms_each": [round(x, 3) for x in ms],
                      "us_per_block": round(med * 1e3 / (S / 64), 4), "digest_ok": ok}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
