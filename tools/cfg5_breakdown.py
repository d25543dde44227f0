#!/usr/bin/env python3
"""Config 5 (BASELINE configs[4]) class by class: where does the mixed stream
lose against the encode headline?

Builds bench.py's Mixed workload and times every class's encode and
reconstruct alone on one stream (HIP events, `--reps` launches each, after one
warm-up), printing one JSON line per (class, op) with the exact algorithmic
bytes of that launch and its rate.

  python tools/cfg5_breakdown.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    import maxio_amd

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    with maxio_amd.Context(device_mask=1, streams_per_device=2) as ctx:
        w = bench.Mixed(torch, ctx, dev, sh, 24 << 30, bench.SEED, streams=1)
        torch.cuda.synchronize()
        tot_ms = tot_b = 0.0
        for (k, m, S, n, t, dl, pres) in w.classes:
            lens = dl + [S] * m

            def enc():
                ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(),
                                          (k + m) * S, S, data_len=dl, stream=sh)

            def dec():
                pr = pres.copy()
                rc, _ = ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, pr,
                                                       shard_len=lens, stream=sh)
                assert rc == 0

            dec_b = 0
            for o in range(n):
                row = pres[o * (k + m): (o + 1) * (k + m)]
                used = [i for i in range(k + m) if row[i]][:k]
                dec_b += sum(lens[i] for i in used) + sum(lens[i] for i in range(k + m) if not row[i])
            for op, fn, nbytes in (("encode", enc, n * (sum(dl) + m * S)), ("reconstruct", dec, dec_b)):
                ms = bench.event_ms(torch, st, fn, a.reps)
                tot_ms += ms
                tot_b += nbytes
                print(json.dumps({"k": k, "m": m, "S": S, "objects": n, "op": op, "ms": round(ms, 4),
                                  "bytes": nbytes, "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}), flush=True)
        print(json.dumps({"sum_ms": round(tot_ms, 3), "bytes": tot_b,
                          "GBps_serial": round(tot_b / (tot_ms * 1e-3) / 1e9, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
