#!/usr/bin/env python3
"""bench.py — device-resident RS encode throughput on MI355X (BASELINE configs[1]).

Step = one pass of the hot path over one batch: Reed–Solomon encode of 1024
objects per GPU, k=4 data + m=2 parity shards of chunk_size = 10 MiB each
(MaxIO `--chunk-size 10485760 --parity-shards 2`, 40 MiB objects), inputs
resident in HBM, parity written to HBM, through the C ABI
(mxec_encode_strided_device) on a dedicated HIP stream.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; objects are partitioned per GPU (weak scaling, no
collective on the data path; only the timing barrier / max-reduce).
Rank 0 prints ONE JSON line.  value = payload GiB/s (k * chunk_size bytes per
object) over all GPUs; roofline = the RS kernel's algorithmic bytes
((k+m) * chunk_size per object) / its HIP-event-timed duration vs 8 TB/s;
cpu_baseline = oracle/ (C restatement of the crate's pure-Rust path) timed on
one host core over a bounded sample.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident RS encode+reconstruct GiB/s (k+m, chunk_size); % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)


def shard_objects(n_total: int, rank: int, world: int) -> range:
    """Objects of the global batch owned by `rank` (contiguous block)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return range(lo, min(n_total, lo + per))


def reduce_max(value: float) -> float:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def cpu_baseline(k: int, m: int, size: int, seconds: float) -> dict:
    """The reference's CPU encode (crate input-major MUL_TABLE lookups,
    restated in oracle/) on one core, over a bounded sample."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/baseline infrastructure only

    rng = np.random.default_rng(0x6D6178696F)
    objs = [[rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)] for _ in range(2)]
    oracle.encode(objs[0], m, size)  # warm tables / page in
    n, t0 = 0, time.perf_counter()
    while True:
        oracle.encode(objs[n % 2], m, size)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {
        "value": round(n * k * size / GIB / el, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n} objects (2 distinct, reused) of k={k} m={m} chunk_size={size} encoded "
                  f"serially in {el:.1f}s by oracle/rs_oracle.c (crate 6.0.0 pure-Rust "
                  f"mul_slice restated: 64 KiB MUL_TABLE, input-major), 1 thread",
    }


def pmc_traffic(config_tag: str):
    """Per-launch HBM bytes of the RS kernel from the committed rocprofv3 PMC
    summary (profiles/*pmc*<tag>*.json), FETCH_SIZE x2 per the gfx950
    correction + WRITE_SIZE, or None."""
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc*{config_tag}*.json"))):
        try:
            with open(p) as f:
                d = json.load(f)
            return d.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)
        except Exception:
            continue
    return None, None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--objects", type=int, default=1024, help="objects per GPU")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--chunk-size", type=int, default=10 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--extra", action="store_true",
                    help="also time the secondary paths (PUT path with SHA-256, config 3 "
                         "reconstruct + verify, copy peak); off by default so a rocprofv3 "
                         "run of the default command profiles only the headline kernel")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import maxio_amd

    ctx = maxio_amd.Context(device_mask=1 << (local if world > 1 else 0), streams_per_device=2)
    k, m, S, n = args.k, args.m, args.chunk_size, args.objects
    objs = shard_objects(n * world, rank, world)
    n_local = len(objs)
    dev = torch.device("cuda", torch.cuda.current_device())

    # Object-major layout in HBM: data [n][k][S], parity [n][m][S].
    g = torch.Generator(device=dev).manual_seed(0x6D6178696F + rank)
    data = torch.empty((n_local, k, S), dtype=torch.uint8, device=dev)
    for o in range(n_local):  # per object keeps the randint temporary small
        data[o].copy_(torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev, generator=g))
    parity = torch.zeros((n_local, m, S), dtype=torch.uint8, device=dev)
    # A dedicated stream: the kernels and the HIP events that time them are
    # on the same queue (a NULL stream would let the library spread calls
    # over its own streams).
    stream = torch.cuda.Stream(device=dev)
    sh = stream.cuda_stream
    torch.cuda.synchronize()

    def step():
        ctx.encode_strided_device(k, m, S, n_local, data.data_ptr(), k * S, S, parity.data_ptr(),
                                  m * S, S, stream=sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # Spot check one object against the oracle (bit-exact) before timing.
    spot_ok = None
    if rank == 0 and S <= (16 << 20):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np
        import oracle

        want = oracle.encode(list(data[0].cpu().numpy()), m, S)
        got = parity[0].cpu().numpy()
        spot_ok = all(np.array_equal(got[i], want[i]) for i in range(m))

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = reduce_max(time.perf_counter() - t0)
    ms_launch = sum(a.elapsed_time(b) for a, b in ev) / len(ev)

    payload = float(n_local * world) * k * S * args.steps  # weak scaling: all ranks
    value = payload / GIB / elapsed
    alg_bytes = float(n_local) * (k + m) * S  # per launch, per GPU
    achieved = alg_bytes / (ms_launch * 1e-3) / 1e9

    extra = None
    if args.extra and rank == 0:
        extra = secondary(ctx, torch, dev, sh, data, parity, k, m, S, n_local)
    # free HBM before the CPU leg
    del data, parity
    torch.cuda.empty_cache()

    if rank == 0:
        traffic, tsrc = pmc_traffic(f"k{k}m{m}")
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: uniform random bytes (torch.randint on device, seeded)",
            "config": {
                "workload": f"RS encode k={k} m={m}, chunk_size={S} B, {n} objects per GPU, "
                            "device-resident (BASELINE configs[1])",
                "k": k, "m": m, "chunk_size": S, "objects_per_gpu": n,
                "payload_bytes_per_step_per_gpu": n_local * k * S,
                "parallelism": "objects partitioned per GPU, no collectives",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "kernel": "rs_apply_fast<R=2,V=4,NT=1>",
                "bytes_per_launch": alg_bytes,
                "ms_per_launch": round(ms_launch, 4),
                "traffic_source": tsrc,
            },
            "cpu_baseline": cpu_baseline(k, m, S, args.cpu_seconds) if args.cpu_seconds > 0 else None,
            "spot_check_vs_oracle": spot_ok,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


def secondary(ctx, torch, dev, sh, data, parity, k, m, S, n_local) -> dict:
    """Reference-equivalent PUT path (encode + SHA-256 of all k+m chunks) on
    the same batch, config 3 (reconstruct 8+4, 2 erasures + verify, 1 MiB,
    8192 data chunks) and the device copy peak.  Reported, not the headline."""
    out = {}
    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    # device copy peak (read + write bytes / time)
    buf = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(buf)
    t = timed(lambda: dst.copy_(buf), 5)
    out["copy_peak_GBps"] = round(2 * buf.numel() / t / 1e9, 1)
    del buf, dst

    dig = torch.empty((n_local, k + m, 32), dtype=torch.uint8, device=dev)

    def put_path():
        ctx.encode_strided_device(k, m, S, n_local, data.data_ptr(), k * S, S, parity.data_ptr(),
                                  m * S, S, digests_ptr=dig.data_ptr(), stream=sh)

    t = timed(put_path, 2)
    out["put_path_encode_plus_sha256"] = {
        "GiBps_payload": round(n_local * k * S / GIB / t, 3), "ms": round(t * 1e3, 2),
        "what": "RS encode + SHA-256 of every data and parity chunk (write_chunk + "
                "compute_and_write_parity compute)"}

    # config 3: k=8 m=4 S=1MiB, 1024 objects (8192 data chunks), 2 data erasures
    import numpy as np

    k3, m3, s3, n3 = 8, 4, 1 << 20, 1024
    g = torch.Generator(device=dev).manual_seed(3)
    obj = torch.randint(0, 256, (n3, k3 + m3, s3), dtype=torch.uint8, device=dev, generator=g)
    dg3 = torch.empty((n3, k3 + m3, 32), dtype=torch.uint8, device=dev)
    ctx.encode_strided_device(k3, m3, s3, n3, obj.data_ptr(), (k3 + m3) * s3, s3,
                              obj[:, k3:].data_ptr(), (k3 + m3) * s3, s3, digests_ptr=dg3.data_ptr(),
                              stream=sh)
    torch.cuda.synchronize()
    rng = np.random.default_rng(0x6D6178696F)
    base_present = np.ones(n3 * (k3 + m3), np.uint8)
    for o in range(n3):
        for i in rng.choice(k3, 2, replace=False):
            base_present[o * (k3 + m3) + i] = 0

    def recon(verify=True):
        pr = base_present.copy()
        rc, _ = ctx.reconstruct_strided_device(k3, m3, s3, n3, obj.data_ptr(), (k3 + m3) * s3, s3, pr,
                                               expected_ptr=dg3.data_ptr() if verify else None,
                                               stream=sh)
        assert rc == 0

    t = timed(recon, 3)
    t_nv = timed(lambda: recon(False), 5)
    out["config3_reconstruct_verify"] = {
        "GiBps_payload": round(n3 * k3 * s3 / GIB / t, 3), "ms": round(t * 1e3, 2),
        "rs_only_ms": round(t_nv * 1e3, 3),
        "rs_only_alg_GBps": round(n3 * (k3 + 2) * s3 / t_nv / 1e9, 1),
        "what": "k=8 m=4 1 MiB: SHA-256 verify of the 10 present shards + rebuild 2, 1024 objects"}
    del obj, dg3, dig
    return out


if __name__ == "__main__":
    sys.exit(main())
