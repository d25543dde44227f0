#!/usr/bin/env python3
"""Is the RS kernel's rate a property of where its batch lands?  Allocates
`--allocs` object-major batches of configs[1]'s shape ([n][k+m][S + pad],
4+2 x 10 MiB, the bench's layout) one after another (most of the card), and
on each, in one process, times with HIP events (median of --reps):

* rs:         the shipping encode (mxec_encode_strided_device), for every
              grid in --grids (workgroups per CU; the lab build's MXEC_RS_BPC)
* pattern:    the RS kernel's own tile / load schedule with XOR math
              (libmaxio_probe mxprobe_rs_pattern_strided)
* f4pattern:  the same bytes at the float4 copy's granularity (one 16-byte
              column per lane, plain loads / stores: mxprobe_rs_float4_strided)
* f4copy:     the guide's float4 copy, first half of the buffer onto the
              second half (the bench's `float4_copy_on_buffers`)

One JSON line per allocation.  Lab tool (needs `make lab`: the default is
MXEC_LIB = the lab build, for MXEC_RS_BPC).

  python tools/placement_lab.py [--objects 256] [--allocs 8] [--grids 1024,512] [--reps 5]
                                [--free-each --spacer-mib 0,4096,...]

--pads-kib sizes the batch for its largest pad, and the other columns
(rs_bpc*, variants, pattern, f4pattern, parts) then run at that stride too;
the rs_pad*k columns are the encode at each listed pad in the same buffer.
--free-each drops each batch before the next (full configs[1] batches, 74 GB,
fit three at a time otherwise); --spacer-mib allocates a spacer of that many
MiB (one value per allocation, cycled) ahead of each batch, so successive
batches land at different places.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MXEC_LIB", os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=256)
    ap.add_argument("--allocs", type=int, default=8)
    ap.add_argument("--grids", default="1024,512")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", action="store_true", help="oracle-check object 0 after the rs timings")
    ap.add_argument("--free-each", action="store_true", help="free each batch before allocating the next")
    ap.add_argument("--spacer-mib", default="", help="comma list: MiB allocated ahead of each batch (cycled)")
    ap.add_argument("--variants", default="",
                    help="semicolon list of name=ENV:val,ENV:val (lab RS knobs, e.g. "
                         "'v2=MXEC_RS_VECS:2;st=MXEC_RS_STORE_NT:0'), each timed like a grid")
    ap.add_argument("--shape", default="4,2,10", help="k,m,chunk MiB (default configs[1]: 4,2,10)")
    ap.add_argument("--base-pad-kib", type=int, default=-1,
                    help="the batch's own shard pad (default: 2112 KiB at chunks >= 4 MiB, else 0, as bench.py)")
    ap.add_argument("--pads-kib", default="",
                    help="comma list of other shard pads (KiB): on every allocation, time rs (first grid) "
                         "with the shards S + pad apart inside the same buffer (the largest pad sizes it)")
    ap.add_argument("--parts", action="store_true",
                    help="also time the RS pattern's halves on each batch (m = 2): reads of the k data shards "
                         "only, writes of the parity only, both; and a plain read stream of the same bytes")
    ap.add_argument("--lds", default="",
                    help="comma list of G:wpc (e.g. 2:512,4:256): the RS pattern with each workgroup's parity held "
                         "in LDS over G tiles and stored in G x 16 KiB runs (mxprobe_rs_pattern_lds, m = 2)")
    ap.add_argument("--revisit", type=int, default=0,
                    help="after the last allocation, time rs (first grid) and f4copy on every kept batch again, "
                         "this many passes (is a slow batch slow for good, or only when it came first?)")
    a = ap.parse_args()
    spacers = [int(x) for x in a.spacer_mib.split(",") if x]
    import torch

    import bench
    import maxio_amd

    k, m, smib = (int(x) for x in a.shape.split(","))
    S, n = smib << 20, a.objects
    pad = (a.base_pad_kib << 10) if a.base_pad_kib >= 0 else ((2 << 20) + (64 << 10) if S >= (4 << 20) else 0)
    pads = [int(x) << 10 for x in a.pads_kib.split(",") if x]
    ss = S + max([pad] + pads)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    sh = st.cuda_stream
    probe = bench.probe_lib()
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    alg = n * (k + m) * S

    def tbps(ms):
        return round(alg / (ms * 1e-3) / 1e12, 4)

    bufs = []
    kept = []  # (alloc index, batch) for --revisit
    for ai in range(a.allocs):
        if a.free_each:
            bufs.clear()
            kept.clear()
            torch.cuda.empty_cache()
        spacer_mib = spacers[ai % len(spacers)] if spacers else 0
        try:
            if spacer_mib:
                bufs.append(torch.empty(spacer_mib << 20, dtype=torch.uint8, device=dev))
            obj = torch.empty((n, k + m, ss), dtype=torch.uint8, device=dev)
        except RuntimeError as e:  # out of memory: stop here
            print(json.dumps({"alloc": ai, "stopped": str(e)[:120]}), flush=True)
            break
        bufs.append(obj)
        kept.append((ai, obj))
        obj[:, :k, :S].random_(0, 256)
        torch.cuda.synchronize()
        d0, p0, ost = obj.data_ptr(), obj[:, k:].data_ptr(), (k + m) * ss
        row = {"alloc": ai, "objects": n, "base_mod_2MiB": d0 % (2 << 20), "spacer_mib": spacer_mib,
               "va_GiB": round(d0 / 2**30, 1)}
        for g in a.grids.split(","):
            os.environ["MXEC_RS_BPC"] = g
            ms = bench.event_ms(torch, st, lambda: ctx.encode_strided_device(
                k, m, S, n, d0, ost, ss, p0, ost, ss, stream=sh), a.reps, warm=2)
            row[f"rs_bpc{g}_TBps"] = tbps(ms)
        os.environ.pop("MXEC_RS_BPC", None)
        for spec in [x for x in a.variants.split(";") if x]:
            name, _, kv = spec.partition("=")
            env = dict(p.split(":", 1) for p in kv.split(",") if p)
            os.environ.update(env)
            ms = bench.event_ms(torch, st, lambda: ctx.encode_strided_device(
                k, m, S, n, d0, ost, ss, p0, ost, ss, stream=sh), a.reps, warm=2)
            for key in env:
                os.environ.pop(key, None)
            row[f"rs_{name}_TBps"] = tbps(ms)
        g0 = a.grids.split(",")[0]
        for pk in pads:
            s2 = S + pk
            os.environ["MXEC_RS_BPC"] = g0
            ms = bench.event_ms(torch, st, lambda: ctx.encode_strided_device(
                k, m, S, n, d0, (k + m) * s2, s2, d0 + k * s2, (k + m) * s2, s2, stream=sh), a.reps, warm=2)
            os.environ.pop("MXEC_RS_BPC", None)
            row[f"rs_pad{pk >> 10}k_TBps"] = tbps(ms)
        if a.check:
            h = obj[0].cpu().numpy()
            want = bench._oracle().encode(list(h[:k, :S]), m, S)
            row["rs_check"] = all((h[k + i, :S] == want[i]).all() for i in range(m))
        row["pattern_TBps"] = tbps(bench.event_ms(torch, st, lambda: probe.mxprobe_rs_pattern_strided(
            d0, p0, k, m, S, n, ost, ost, ss, sh), a.reps))
        row["f4pattern_TBps"] = tbps(bench.event_ms(torch, st, lambda: probe.mxprobe_rs_float4_strided(
            d0, p0, k, m, S, n, ost, ost, ss, sh), a.reps))
        for spec in [x for x in a.lds.split(",") if x]:
            G, wpc = (int(x) for x in spec.split(":"))
            probe.mxprobe_rs_pattern_lds.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                     ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            probe.mxprobe_rs_pattern_lds.restype = ctypes.c_int
            rc = probe.mxprobe_rs_pattern_lds(d0, p0, k, S, n, ost, ss, G, wpc, sh)
            if rc:
                raise SystemExit(f"mxprobe_rs_pattern_lds rc {rc}")
            row[f"pattern_lds{G}_wpc{wpc}_TBps"] = tbps(bench.event_ms(torch, st, lambda: probe.mxprobe_rs_pattern_lds(
                d0, p0, k, S, n, ost, ss, G, wpc, sh), a.reps))
        if a.parts:
            sink = torch.zeros(16, dtype=torch.uint8, device=dev)
            probe.mxprobe_rs_pattern_part.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                      ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                      ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
            probe.mxprobe_rs_pattern_part.restype = ctypes.c_int
            for part, name, nbytes in ((0, "reads", k * S * n), (1, "writes", m * S * n), (2, "both", (k + m) * S * n)):
                ms = bench.event_ms(torch, st, lambda: probe.mxprobe_rs_pattern_part(
                    d0, p0, k, S, n, ost, ss, part, sink.data_ptr(), sh), a.reps)
                row[f"part_{name}_TBps"] = round(nbytes / (ms * 1e-3) / 1e12, 4)
            rb = (obj.numel() * k // (k + m)) & ~15
            ms = bench.event_ms(torch, st, lambda: probe.mxprobe_read(d0, rb, sink.data_ptr(), sh), a.reps)
            row["read_stream_TBps"] = round(rb / (ms * 1e-3) / 1e12, 4)
        half = (obj.numel() // 2) & ~15
        ms = bench.event_ms(torch, st, lambda: probe.mxprobe_copy_float4(d0 + half, d0, half, sh), a.reps)
        row["f4copy_TBps"] = round(2 * half / (ms * 1e-3) / 1e12, 4)
        for key in [x for x in row if x.startswith(("rs_", "pattern")) and x.endswith("_TBps")]:
            row[key.replace("_TBps", "_of_f4copy")] = round(row[key] / row["f4copy_TBps"], 4)
        print(json.dumps(row), flush=True)
    g0 = a.grids.split(",")[0]
    for rp in range(a.revisit):
        for ai, obj in kept:
            d0, p0, ost = obj.data_ptr(), obj[:, k:].data_ptr(), (k + m) * ss
            os.environ["MXEC_RS_BPC"] = g0
            row = {"revisit": rp, "alloc": ai}
            row[f"rs_bpc{g0}_TBps"] = tbps(bench.event_ms(torch, st, lambda: ctx.encode_strided_device(
                k, m, S, n, d0, ost, ss, p0, ost, ss, stream=sh), a.reps, warm=2))
            os.environ.pop("MXEC_RS_BPC", None)
            half = (obj.numel() // 2) & ~15
            ms = bench.event_ms(torch, st, lambda: probe.mxprobe_copy_float4(d0 + half, d0, half, sh), a.reps)
            row["f4copy_TBps"] = round(2 * half / (ms * 1e-3) / 1e12, 4)
            row[f"rs_bpc{g0}_of_f4copy"] = round(row[f"rs_bpc{g0}_TBps"] / row["f4copy_TBps"], 4)
            print(json.dumps(row), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
