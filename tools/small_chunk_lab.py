#!/usr/bin/env python3
"""Why do config 5's small-chunk classes run below the big ones?

Times encode_strided_device (HIP events, after one warm-up) on ~1.6 GB
batches of k+m shards at several chunk sizes, with every data chunk whole and
with a short last chunk (the config 5 shape: one length boundary per object,
its tile taking the edge path), so the two costs -- per-tile overhead and the
edge path -- separate.

  python tools/small_chunk_lab.py [--reps 10] [--km 8,4]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--km", default="8,4")
    ap.add_argument("--budget", type=int, default=1638 << 20)
    a = ap.parse_args()
    import torch

    import bench
    import maxio_amd

    k, m = (int(x) for x in a.km.split(","))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    with maxio_amd.Context(device_mask=1, streams_per_device=2) as ctx:
        for S in (64 << 10, 256 << 10, 1 << 20, 10 << 20):
            n = max(1, a.budget // ((k + m) * S))
            t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device=dev)
            for label, last in (("whole", S), ("short_last", S // 2 + 4321)):
                dl = [S] * (k - 1) + [last]
                nbytes = n * (sum(dl) + m * S)

                def enc():
                    ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(),
                                              (k + m) * S, S, data_len=dl, stream=sh)

                ms = bench.event_ms(torch, st, enc, a.reps)
                print(json.dumps({"k": k, "m": m, "S": S, "objects": n, "chunks": label, "ms": round(ms, 4),
                                  "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}), flush=True)
            del t
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
