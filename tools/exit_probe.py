#!/usr/bin/env python3
"""Which step of a libmaxio_ec process trips rocprofv3's exit-time fault?

Under `rocprofv3 --kernel-trace --memory-copy-trace`, `bench.py` printed its
line and then died with SIGSEGV inside libhsa-runtime64.so, called from
librocprofiler-sdk.so during the profiler tool's own __cxa_finalize
(profiles/r5/trace_bench_exit_crash.err, resolved with BENCH_DUMP_MAPS=1); a
torch-only program under the same options exits 0.  This runs one small
piece of the library's work and exits, so a series of runs under the
profiler narrows the trigger:

  python tools/exit_probe.py <what> [--no-close]
    what: open          mxec_open / mxec_close only
          device        + one device-resident encode (a kernel launch)
          host_pinned   + one mxec_encode_batch_host from mxec_host_alloc memory
          host_pageable + one mxec_encode_batch_host from pageable memory
          hash          + one mxec_sha256_batch (host pointers)
          torch_copy    no mxec call after open: torch's own pinned H2D / D2H
                        copies on a side stream (does any async copy arm it?)
          torch_pageable no mxec call after open: torch's H2D / D2H copies of
                        pageable memory (HIP stages them itself)
          attr_pageable no mxec work after open: hipPointerGetAttributes on a
                        pageable buffer (what is_pinned() asks of every
                        pageable shard), its error cleared
          torch_streams torch alone on eight streams (more than the four
                        hardware queues HIP gives a process), each with a
                        pinned H2D copy, a kernel and a D2H copy
  --no-close leaves the context open at exit (no stream / event teardown).
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["open", "device", "host_pinned", "host_pageable", "hash", "torch_copy",
                                        "torch_pageable", "attr_pageable", "torch_streams"])
    ap.add_argument("--no-close", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch

    import maxio_amd

    torch.cuda.set_device(0)
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    k, m, S, n = 4, 2, 1 << 20, 16
    if a.what == "device":
        t = torch.randint(0, 256, (n, k + m, S), dtype=torch.uint8, device="cuda")
        ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(), (k + m) * S, S)
        torch.cuda.synchronize()
    elif a.what in ("host_pinned", "host_pageable"):
        if a.what == "host_pinned":
            data = ctx.host_array(n * k * S).reshape(n, k, S)
            par = ctx.host_array(n * m * S).reshape(n, m, S)
        else:
            data = np.zeros((n, k, S), np.uint8)
            par = np.zeros((n, m, S), np.uint8)
        data[:] = 7
        dig = np.zeros(n * (k + m) * 32, np.uint8)
        ctx.encode_batch_host([(k, m, S)] * n, [data[o, j].ctypes.data for o in range(n) for j in range(k)],
                              [par[o, i].ctypes.data for o in range(n) for i in range(m)], digests=dig)
        if a.what == "host_pinned":
            ctx.host_free(data)
            ctx.host_free(par)
    elif a.what == "torch_copy":
        h = torch.empty(64 << 20, dtype=torch.uint8).pin_memory()
        h.fill_(7)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            d = h.to("cuda", non_blocking=True)
            back = torch.empty_like(h).pin_memory()
            back.copy_(d, non_blocking=True)
        s.synchronize()
        assert int(back[12345]) == 7
    elif a.what == "torch_pageable":
        h = torch.full((64 << 20,), 7, dtype=torch.uint8)  # pageable
        d = h.to("cuda")
        back = d.cpu()
        assert int(back[12345]) == 7
    elif a.what == "attr_pageable":
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        buf = np.zeros(1 << 20, np.uint8)  # pageable
        attr = ctypes.create_string_buffer(512)  # hipPointerAttribute_t (smaller)
        rc = hip.hipPointerGetAttributes(attr, ctypes.c_void_p(buf.ctypes.data))
        hip.hipGetLastError()
        print(f"hipPointerGetAttributes(pageable) = {rc}", flush=True)
    elif a.what == "torch_streams":
        ss = [torch.cuda.Stream() for _ in range(8)]
        hs = [torch.full((8 << 20,), j, dtype=torch.uint8).pin_memory() for j in range(8)]
        outs = []
        for j, s in enumerate(ss):
            with torch.cuda.stream(s):
                d = hs[j].to("cuda", non_blocking=True)
                d.add_(1)
                back = torch.empty_like(hs[j]).pin_memory()
                back.copy_(d, non_blocking=True)
                outs.append(back)
        for s in ss:
            s.synchronize()
        assert all(int(o[777]) == j + 1 for j, o in enumerate(outs))
    elif a.what == "hash":
        ctx.sha256([bytes(range(256)) * 4096] * 8)
    if not a.no_close:
        ctx.close()
    print(f"exit_probe {a.what} close={not a.no_close}: done", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
