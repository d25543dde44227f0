#!/usr/bin/env python3
"""Host-side cost of one headline encode call (bench.py config 2): how long
encode_strided_device takes to return while the GPU runs the previous
launches, per call, over 30 calls -- the host must stay ahead of a ~10.5 ms
kernel for the step time to be the kernel time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch

    import bench
    import maxio_amd

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    with maxio_amd.Context(device_mask=1, streams_per_device=2) as ctx:
        w = bench.make_workload("2", torch, ctx, dev, st.cuda_stream, 0, 0)
        torch.cuda.synchronize()
        for _ in range(3):
            w.step()
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for _ in range(30):
            t = time.perf_counter()
            w.step()
            host.append((time.perf_counter() - t) * 1e3)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"host_ms_per_call": [round(x, 3) for x in host],
                          "enqueue_all_ms": round((t1 - t0) * 1e3, 2),
                          "wall_ms_per_step": round((t2 - t0) * 1e3 / 30, 3)}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
