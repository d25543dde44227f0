#!/usr/bin/env python3
"""Is HBM write bandwidth a property of the physical region?  Allocates
`--chunks` buffers of `--gib` GiB each in order (most of the card), then
times a nontemporal write stream, a read stream and a copy into each chunk
(the probe kernels of libmaxio_probe.so, HIP events, median of --reps), and
prints one line per chunk in allocation order.  The round-2 allocation
study (profiles/r2_cfg2_allocation_spread.txt) saw writes into some
allocations run at 4.7-4.8 TB/s and into others at 5.6-6.3 while reads
stayed at 6.2-6.6.

  python tools/region_lab.py [--gib 8] [--chunks 30] [--reps 5]
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
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--policies", action="store_true",
                    help="per chunk: write streams and the RS access pattern (k=4 m=2, 1 MiB shards, "
                         "object-major) under each store policy: 0 nt, 1 plain, 2 sc1, 3 sc0 sc1, 4 sc1 nt")
    a = ap.parse_args()
    import torch

    import bench

    probe = bench.probe_lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    sh = st.cuda_stream
    n = a.gib << 30
    sink = torch.zeros(16, dtype=torch.uint8, device=dev)

    def timed(fn):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        torch.cuda.synchronize()
        for e0, e1 in ev:
            e0.record(st)
            assert fn() == 0
            e1.record(st)
        torch.cuda.synchronize()
        return sorted(e0.elapsed_time(e1) for e0, e1 in ev)[a.reps // 2]

    bufs = []
    for i in range(a.chunks):
        try:
            bufs.append(torch.empty(n, dtype=torch.uint8, device=dev))
        except RuntimeError:
            break
    free, total = torch.cuda.mem_get_info()
    print(json.dumps({"chunks": len(bufs), "gib_each": a.gib, "free_GiB": round(free / 2**30, 1),
                      "total_GiB": round(total / 2**30, 1)}), flush=True)
    half = n // 2
    if a.policies:
        import ctypes

        probe.mxprobe_rs_pattern_policy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        probe.mxprobe_rs_pattern_policy.restype = ctypes.c_int
        k, m, S = 4, 2, 1 << 20
        nobj = n // ((k + m) * S)
        for i, b in enumerate(bufs):
            row = {"chunk": i}
            for pol, name in enumerate(("nt", "plain", "sc1", "sc0sc1", "sc1nt")):
                w = timed(lambda: probe.mxprobe_write(b.data_ptr(), n, pol, sh))
                pt = timed(lambda: probe.mxprobe_rs_pattern_policy(b.data_ptr(), b.data_ptr() + k * S, k, S, nobj,
                                                                   (k + m) * S, S, pol, sh))
                row[f"write_{name}"] = round(n / w / 1e9, 3)
                row[f"rs_{name}"] = round(nobj * (k + m) * S / pt / 1e9, 3)
            print(json.dumps(row), flush=True)
        return 0
    for i, b in enumerate(bufs):
        w = timed(lambda: probe.mxprobe_write(b.data_ptr(), n, 0, sh))
        wp = timed(lambda: probe.mxprobe_write(b.data_ptr(), n, 1, sh))
        r = timed(lambda: probe.mxprobe_read(b.data_ptr(), n, sink.data_ptr(), sh))
        c = timed(lambda: probe.mxprobe_copy(b.data_ptr() + half, b.data_ptr(), half, sh))
        print(json.dumps({"chunk": i, "va_GiB": round((b.data_ptr() - bufs[0].data_ptr()) / 2**30, 2),
                          "write_nt_TBps": round(n / w / 1e9, 3), "write_plain_TBps": round(n / wp / 1e9, 3),
                          "read_TBps": round(n / r / 1e9, 3), "copy_TBps": round(2 * half / c / 1e9, 3)}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
