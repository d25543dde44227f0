#!/usr/bin/env python3
"""Where config 5 loses against config 2: per (k, m, S) class, the encode
rate of the uniform kernel (mxec_encode_strided_device, one class per call)
and of the grouped kernel (the same class through mxec_encode_batch_device
beside a one-object decoy of another shape, so the call is not uniform), with
full and short last chunks.  HIP-event timed on one stream; algorithmic bytes
counted exactly (k data chunks as they are + m parity).

  python tools/mixed_lab.py [--budget-gib 1.6] [--reps 5]
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
    ap.add_argument("--budget-gib", type=float, default=1.6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kms", default="4:2,8:4")
    ap.add_argument("--sizes", default="65536,262144,1048576,4194304,10485760")
    a = ap.parse_args()
    import numpy as np
    import torch

    import maxio_amd
    from maxio_amd import _native as N

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sh = st.cuda_stream
    rng = np.random.default_rng(7)

    def timed(fn):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        torch.cuda.synchronize()
        for e0, e1 in ev:
            e0.record(st)
            fn()
            e1.record(st)
        torch.cuda.synchronize()
        return sorted(e0.elapsed_time(e1) for e0, e1 in ev)[a.reps // 2]

    decoy = torch.zeros((1, 3, 4096), dtype=torch.uint8, device=dev)
    with maxio_amd.Context(device_mask=1, streams_per_device=1) as ctx:
        for km in a.kms.split(","):
            k, m = map(int, km.split(":"))
            for S in map(int, a.sizes.split(",")):
                n = max(1, int(a.budget_gib * (1 << 30)) // ((k + m) * S))
                t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device=dev)
                for short in (False, True):
                    last = int(rng.integers(1, S)) if short else S
                    dl = [S] * (k - 1) + [last]
                    alg = n * (sum(dl) + m * S)
                    base = t.data_ptr()
                    ms_u = timed(lambda: ctx.encode_strided_device(k, m, S, n, base, (k + m) * S, S,
                                                                   base + k * S, (k + m) * S, S, data_len=dl,
                                                                   stream=sh))
                    objs = [N.Object(k, m, S)] * n + [N.Object(2, m, 4096)]
                    dp, pp, ln = [], [], []
                    for o in range(n):
                        dp += [base + o * (k + m) * S + j * S for j in range(k)]
                        pp += [base + o * (k + m) * S + (k + i) * S for i in range(m)]
                        ln += dl
                    dp += [decoy[0, 0].data_ptr(), decoy[0, 1].data_ptr()]
                    pp += [decoy[0, 2].data_ptr()] * m  # the decoy's outputs may alias: timing only
                    ln += [4096, 4096]
                    arr = (N.Object * len(objs))(*objs)
                    dpa = (ctypes.c_void_p * len(dp))(*dp)
                    ppa = (ctypes.c_void_p * len(pp))(*pp)
                    lna = (ctypes.c_uint64 * len(ln))(*ln)
                    ms_g = timed(lambda: ctx.encode_batch_device(arr, dpa, ppa, data_len=lna, stream=sh))
                    print(json.dumps({"k": k, "m": m, "S": S, "n": n, "short_last": short,
                                      "uniform_TBps": round(alg / ms_u / 1e9, 3),
                                      "grouped_TBps": round(alg / ms_g / 1e9, 3),
                                      "uniform_ms": round(ms_u, 4), "grouped_ms": round(ms_g, 4)}), flush=True)
                del t
                torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
