"""Where a single GET's time goes (tools/e2e_get_bench.py reports ~45 ms for
one 8 x 1 MiB object against ~30 ms of SHA-256 chain): time each stage of
the path on its own.

  device_sha[n x L]  mxec_sha256_batch_device on n device-resident messages
                     (the kernel alone, caller's stream, synchronised)
  host_sha[8 x 1MiB] mxec_sha256_batch: pageable H2D + combiner + D2H
  file_reads         the 8 shard files read into host memory (Python)
  get                mxec_get_object_chunked of the whole object

Medians of --reps runs; one JSON line."""
import argparse, json, os, statistics, sys, tempfile, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(f, reps):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return round(statistics.median(ts) * 1e3, 3)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import maxio_amd

    ctx = maxio_amd.Context(streams_per_device=2)
    out = {"what": "single-GET stage latencies, ms (median)"}
    S = 1 << 20
    dev = torch.randint(0, 256, (512 * S,), dtype=torch.uint8, device="cuda")
    dig = torch.empty(512 * 32, dtype=torch.uint8, device="cuda")
    base = dev.data_ptr()
    for n, L in ((1, S), (8, S), (64, S), (512, S), (8, 64 << 10), (8, 4096)):
        ptrs = [base + i * S for i in range(n)]

        def f():
            ctx.sha256_batch_device(ptrs, [L] * n, dig.data_ptr())
            torch.cuda.synchronize()
        ms = med(f, args.reps)
        blocks = (L + 9 + 63) // 64
        out[f"device_sha_{n}x{L}"] = {"ms": ms, "us_per_block": round(ms * 1e3 / blocks, 3)}
    rng = np.random.default_rng(3)
    body = rng.integers(0, 256, 8 * S, dtype=np.uint8)
    bufs = [body[i * S:(i + 1) * S] for i in range(8)]
    out["host_sha_8x1MiB"] = {"ms": med(lambda: ctx.sha256(bufs), args.reps)}
    d = tempfile.mkdtemp(prefix="mxec_lat_")
    ec = os.path.join(d, "obj.ec")
    ctx.put_object_chunked(ec, S, 4, body)
    files = [os.path.join(ec, f"{i:06}") for i in range(8)]

    def reads():
        for p in files:
            with open(p, "rb") as fh:
                fh.read()
    out["file_reads_8x1MiB"] = {"ms": med(reads, args.reps)}
    out["get_8x1MiB"] = {"ms": med(lambda: ctx.get_object_chunked(ec), args.reps)}
    out["put_8x1MiB"] = {"ms": med(lambda: ctx.put_object_chunked(ec, S, 4, body), args.reps)}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
