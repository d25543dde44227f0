#!/usr/bin/env python3
"""End-to-end PUT-path rate from host memory (DESIGN.md §5 "end to end").

Objects start in host memory (the request body) and parity chunks + digests
end in host memory, through mxec_encode_batch_host: H2D, RS encode, SHA-256 of
every chunk, D2H, pipelined over streams with the batch resident in HBM.
Reports payload GiB/s (k * chunk_size per object) for pinned and pageable
host buffers, with and without the SHA-256 digests, next to the raw PCIe
H2D / D2H copy rates of the same box.

  python tools/e2e_bench.py [--objects 256] [--k 4 --m 2 --chunk-size 10485760]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def fill(buf: np.ndarray, seed: int) -> None:
    """Random bytes without generating gigabytes of randomness: tile a 64 MiB block."""
    blk = np.random.default_rng(seed).integers(0, 256, 64 << 20, dtype=np.uint8)
    flat = buf.reshape(-1)
    for o in range(0, flat.size, blk.size):
        n = min(blk.size, flat.size - o)
        flat[o:o + n] = blk[:n]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=256)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--chunk-size", type=int, default=10 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--alloc", choices=["torch", "mxec"], default="torch",
                    help="page-locked buffers from torch pin_memory (SDMA always) or mxec_host_alloc "
                         "(mapped: MXEC_PIPE_COPY decides SDMA or CU-wave copies)")
    ap.add_argument("--modes", default="pinned,pageable")
    ap.add_argument("--get", action="store_true",
                    help="also time the GET side: mxec_reconstruct_batch_host over the same objects with two "
                         "erased shards each, without and with verification of the present shards")
    args = ap.parse_args()

    import torch

    import maxio_amd

    k, m, S, n = args.k, args.m, args.chunk_size, args.objects
    ctx = maxio_amd.Context(streams_per_device=2)
    out = {"what": "end-to-end PUT compute from host memory (mxec_encode_batch_host)",
           "k": k, "m": m, "chunk_size": S, "objects": n, "devices": ctx.device_ids()}

    # raw PCIe rates (one 1 GiB pinned buffer)
    hb = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    db = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for name, fn in (("h2d", lambda: db.copy_(hb, non_blocking=True)),
                     ("d2h", lambda: hb.copy_(db, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        out[f"pcie_{name}_GBps"] = round(5 * (1 << 30) / (time.perf_counter() - t0) / 1e9, 1)
    # both directions at once on two streams: do H2D and D2H overlap?
    hb2 = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    db2 = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        with torch.cuda.stream(s1):
            db.copy_(hb, non_blocking=True)
        with torch.cuda.stream(s2):
            hb2.copy_(db2, non_blocking=True)
    torch.cuda.synchronize()
    out["pcie_bidir_GBps_total"] = round(10 * (1 << 30) / (time.perf_counter() - t0) / 1e9, 1)
    del hb, db, hb2, db2

    objs = [(k, m, S)] * n
    out["alloc"] = args.alloc
    out["MXEC_PIPE_COPY"] = os.environ.get("MXEC_PIPE_COPY", "auto")
    for mode in args.modes.split(","):
        if mode == "pinned" and args.alloc == "mxec":
            data = ctx.host_array(n * k * S).reshape(n, k, S)
            par = ctx.host_array(n * m * S).reshape(n, m, S)
        elif mode == "pinned":
            data_t = torch.empty((n, k, S), dtype=torch.uint8).pin_memory()
            par_t = torch.empty((n, m, S), dtype=torch.uint8).pin_memory()
            data, par = data_t.numpy(), par_t.numpy()
        else:
            data = np.empty((n, k, S), np.uint8)
            par = np.empty((n, m, S), np.uint8)
        fill(data, 7)
        dptr = [data[o, j].ctypes.data for o in range(n) for j in range(k)]
        pptr = [par[o, i].ctypes.data for o in range(n) for i in range(m)]
        dig_keep = None
        for sha in (True, False):
            dig = np.zeros(n * (k + m) * 32, np.uint8) if sha else None
            if sha:
                dig_keep = dig
            ctx.encode_batch_host(objs, dptr, pptr, digests=dig)  # warm (pool, tables)
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ctx.encode_batch_host(objs, dptr, pptr, digests=dig)
            el = (time.perf_counter() - t0) / args.reps
            key = f"{mode}_{'rs_sha' if sha else 'rs_only'}"
            out[key] = {"s": round(el, 4), "GiBps_payload": round(n * k * S / GIB / el, 2)}
        if args.get:
            sptr = []
            for o in range(n):
                sptr += [data[o, j].ctypes.data for j in range(k)] + [par[o, i].ctypes.data for i in range(m)]
            rng = np.random.default_rng(11)
            present0 = np.ones(n * (k + m), np.uint8)
            for o in range(n):
                for i in rng.choice(k + m, 2, replace=False):
                    present0[o * (k + m) + i] = 0
            for verify in (False, True):
                exp = dig_keep if verify else None
                rc, _ = ctx.reconstruct_batch_host(objs, sptr, present0.copy(), expected=exp)  # warm
                assert rc == 0, rc
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    rc, _ = ctx.reconstruct_batch_host(objs, sptr, present0.copy(), expected=exp)
                    assert rc == 0, rc
                el = (time.perf_counter() - t0) / args.reps
                out[f"{mode}_get_{'verify' if verify else 'rs_only'}"] = {
                    "s": round(el, 4), "GiBps_payload": round(n * k * S / GIB / el, 2)}
        # spot check one object against the oracle
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        want = oracle.encode(list(data[n // 2]), m, S)
        out[f"{mode}_spot_check"] = all(np.array_equal(par[n // 2, i], want[i]) for i in range(m))
        del data, par
    print(json.dumps(out), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
