#!/usr/bin/env python3
"""Run-to-run spread of the headline encode: is it the allocation?

The same binary on the same box measured config 2 at 3 235-3 719 GiB/s from
one process to the next (profiles/r2_cfg2_spread.txt) while launches inside a
process vary by < 1 %.  This re-allocates the 40 GiB data + 20 GiB parity
tensors `--allocs` times in ONE process and times `--reps` launches on each
allocation, so a spread that follows the allocation shows up here.

  python tools/alloc_lab.py [--allocs 6] [--reps 5] [--objects 1024]
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
    ap.add_argument("--allocs", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--objects", type=int, default=1024)
    ap.add_argument("--alloc", default="torch", choices=["torch", "contiguous"],
                    help="torch: the caching allocator (hipMalloc); contiguous: "
                         "hipExtMallocWithFlags(hipDeviceMallocContiguous)")
    ap.add_argument("--layout", default="separate", choices=["separate", "parity_first", "object_major"],
                    help="separate: data [n][k][S] then parity [n][m][S] (the bench); parity_first: the "
                         "same, parity allocated first; object_major: one [n][k+m][S] tensor, each object's "
                         "parity after its data")
    ap.add_argument("--pad", type=int, default=0,
                    help="object_major only: bytes of padding after each shard (shard stride S + pad)")
    a = ap.parse_args()
    import torch

    import maxio_amd

    k, m, S, n = 4, 2, 10 << 20, a.objects
    dev = torch.device("cuda", 0)
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]

    class Raw:
        """Device bytes from hipExtMallocWithFlags, seen by torch zero-copy."""

        def __init__(self, nbytes):
            self.p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(self.p), nbytes, 0x4)  # hipDeviceMallocContiguous
            assert rc == 0, f"hipExtMallocWithFlags rc={rc}"
            self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                             "data": (self.p.value, False), "version": 3}

        def free(self):
            hip.hipFree(self.p)

    def alloc(shape):
        if a.alloc == "torch":
            return torch.empty(shape, dtype=torch.uint8, device=dev), None
        nb = 1
        for x in shape:
            nb *= x
        r = Raw(nb)
        return torch.as_tensor(r, device=dev).view(shape), r
    st = torch.cuda.Stream()
    sys.path.insert(0, ROOT)
    import bench

    probe = bench.probe_lib()
    sink = torch.zeros(16, dtype=torch.uint8, device=dev)

    def timed(fn, reps):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        torch.cuda.synchronize()
        for e0, e1 in ev:
            e0.record(st)
            fn()
            e1.record(st)
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) for e0, e1 in ev]

    with maxio_amd.Context(device_mask=1, streams_per_device=2) as ctx:
        for i in range(a.allocs):
            rdat = rp = None
            sstride = S
            if a.layout == "object_major":
                sstride = S + a.pad
                whole, rdat = alloc((n, k + m, sstride))
                whole.random_(0, 256)
                data, parity = whole[:, :k], whole[:, k:]
                dstride = pstride = (k + m) * sstride
            else:
                if a.layout == "parity_first":
                    parity, rp = alloc((n, m, S))
                    data, rdat = alloc((n, k, S))
                else:
                    data, rdat = alloc((n, k, S))
                    parity, rp = alloc((n, m, S))
                data.random_(0, 256)
                dstride, pstride = k * S, m * S
            torch.cuda.synchronize()

            def step():
                ctx.encode_strided_device(k, m, S, n, data.data_ptr(), dstride, sstride, parity.data_ptr(), pstride,
                                          sstride, stream=st.cuda_stream)

            ms = timed(step, a.reps)
            alg = n * (k + m) * S
            # the same buffers under the probe streams: the RS pattern with XOR,
            # a read of the data, a copy of the parity-sized front of the data
            # into the parity (write side)
            if a.layout == "object_major":
                print(json.dumps({"alloc": i, "layout": a.layout, "pad": a.pad, "ms": [round(x, 3) for x in ms],
                                  "rs_TBps": round(alg / (sum(ms) / len(ms) * 1e-3) / 1e12, 3)}), flush=True)
                del data, parity, whole
                if rdat is not None:
                    rdat.free()
                torch.cuda.empty_cache()
                continue
            pat = timed(lambda: probe.mxprobe_rs_pattern(data.data_ptr(), parity.data_ptr(), k, m, S, n,
                                                         st.cuda_stream), 3)
            rd = timed(lambda: probe.mxprobe_read(data.data_ptr(), n * k * S, sink.data_ptr(), st.cuda_stream), 3)
            cp = timed(lambda: probe.mxprobe_copy(parity.data_ptr(), data.data_ptr(), n * m * S, st.cuda_stream), 3)
            wnt = timed(lambda: probe.mxprobe_write(parity.data_ptr(), n * m * S, 0, st.cuda_stream), 3)
            wpl = timed(lambda: probe.mxprobe_write(parity.data_ptr(), n * m * S, 1, st.cuda_stream), 3)
            wdn = timed(lambda: probe.mxprobe_write(data.data_ptr(), n * m * S, 0, st.cuda_stream), 3)
            avg = lambda v: sum(v) / len(v)
            print(json.dumps({"alloc": i, "how": a.alloc, "layout": a.layout, "ms": [round(x, 3) for x in ms],
                              "rs_TBps": round(alg / (avg(ms) * 1e-3) / 1e12, 3),
                              "pattern_TBps": round(alg / (avg(pat) * 1e-3) / 1e12, 3),
                              "read_data_TBps": round(n * k * S / (avg(rd) * 1e-3) / 1e12, 3),
                              "copy_into_parity_TBps": round(2 * n * m * S / (avg(cp) * 1e-3) / 1e12, 3),
                              "write_parity_nt_TBps": round(n * m * S / (avg(wnt) * 1e-3) / 1e12, 3),
                              "write_parity_plain_TBps": round(n * m * S / (avg(wpl) * 1e-3) / 1e12, 3),
                              "write_data_front_nt_TBps": round(n * m * S / (avg(wdn) * 1e-3) / 1e12, 3)}),
                  flush=True)
            torch.cuda.synchronize()
            del data, parity
            for r in (rdat, rp):
                if r is not None:
                    r.free()
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
