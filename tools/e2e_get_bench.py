#!/usr/bin/env python3
"""End-to-end PUT and GET rates through the file layer.

The GET path starts at the shard files `{key}.ec/{i:06}` + manifest.json and
ends in a host buffer (VerifiedChunkReader, chunk_reader.rs:35-276): read each
chunk, SHA-256 verify against the manifest, rebuild bad chunks from parity.
Objects are written with mxec_put_object_chunked into a scratch directory
(so the reads below come from the page cache: the rate is the path's, not
the disk's), then read back with mxec_get_object_chunked by W host threads
(concurrent requests on tokio workers), healthy and degraded (erasures
deleted from disk).  Beside it the reference algorithm on the host cores:
read the files, hashlib.sha256 per chunk (OpenSSL, SHA-NI like sha2 0.10),
and for every bad chunk try_reconstruct_data_chunk (oracle/, the crate's
algorithm) over all k+m shard files, as chunk_reader.rs:157-226 does.

  python tools/e2e_get_bench.py [--objects 128 --k 8 --chunk-size 1048576 --parity 4 --threads 16]
"""
from __future__ import annotations

import argparse
import threading
import ctypes
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def reference_get(ec_dir: str, oracle) -> int:
    """chunk_reader.rs semantics on the host: verify every data chunk, rebuild
    the bad ones from all k+m shards.  Returns bytes served."""
    with open(os.path.join(ec_dir, "manifest.json")) as f:
        man = json.load(f)
    k = man["chunk_count"]
    m = man.get("parity_shards") or 0
    S = man.get("shard_size") or man["chunk_size"]
    chunks = man["chunks"]
    served = 0
    for i in range(k):
        p = os.path.join(ec_dir, f"{i:06}")
        ok = False
        if os.path.exists(p):
            with open(p, "rb") as f:
                data = f.read()
            ok = len(data) == chunks[i]["size"] and hashlib.sha256(data).hexdigest() == chunks[i]["sha256"]
        if not ok:
            shards, exp = [], []
            for j in range(k + m):
                q = os.path.join(ec_dir, f"{j:06}")
                shards.append(open(q, "rb").read() if os.path.exists(q) else None)
                exp.append(bytes.fromhex(chunks[j]["sha256"]))
            data, rc, _ = oracle.try_reconstruct_data_chunk(shards, k, m, S, exp,
                                                            [c["size"] for c in chunks], i)
            assert rc == 0, rc
        served += len(data)
    return served


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--chunk-size", type=int, default=1 << 20)
    ap.add_argument("--parity", type=int, default=4)
    ap.add_argument("--erasures", type=int, default=2)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-objects", type=int, default=32)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--pinned", action="store_true",
                    help="PUT bodies and GET buffers in page-locked memory (mxec_host_alloc)")
    args = ap.parse_args()

    import maxio_amd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # baseline only

    k, S, m, n = args.k, args.chunk_size, args.parity, args.objects
    size = k * S
    base = tempfile.mkdtemp(prefix="mxec_get_", dir=args.dir)
    out = {"what": "GET end to end (page-cached shard files -> verified host buffer)",
           "k": k, "m": m, "chunk_size": S, "object_bytes": size, "objects": n,
           "threads": args.threads, "scratch": base, "host_cpus_allowed": len(os.sched_getaffinity(0))}
    try:
        ctx = maxio_amd.Context(streams_per_device=args.threads)
        rng = np.random.default_rng(7)
        block = rng.integers(0, 256, size + 4096, dtype=np.uint8)
        if args.pinned:
            pb = ctx.host_array(block.size)
            pb[:] = block
            block = pb
        out["pinned_buffers"] = bool(args.pinned)
        dirs = [os.path.join(base, f"obj{o}.ec") for o in range(n)]
        lib0 = maxio_amd.lib()

        def gpu_put(o):
            body = block[o % 4096: o % 4096 + size]
            rc = lib0.mxec_put_object_chunked(ctx.handle, dirs[o].encode(), S, m, body.ctypes.data, size)
            assert rc == 0, rc
            return size

        # PUT (put_object_chunked: chunk files + parity + manifest.json, SHA-256
        # of every chunk), W threads; the first pass writes, the timed pass
        # overwrites the same files.
        with ThreadPoolExecutor(args.threads) as pool:
            list(pool.map(gpu_put, range(n)))
            c0 = os.times()
            t = time.perf_counter()
            total = sum(pool.map(gpu_put, range(n)))
            el = time.perf_counter() - t
            c1 = os.times()
        out["gpu_put"] = {"GiBps": round(total / GIB / el, 3), "s": round(el, 4),
                          "host_cores_busy": round((c1.user + c1.system - c0.user - c0.system) / el, 2)}

        def host_write(o):
            """The file writes of a PUT alone (k data + m parity-sized chunk
            files, rewritten in place as the timed PUT pass does): what the
            filesystem can take."""
            body = block[o % 4096: o % 4096 + size]
            for i in range(k + m):
                with open(os.path.join(dirs[o], f"{i:06}"), "wb") as f:
                    f.write(body[(i % k) * S:(i % k + 1) * S])
            return size

        with ThreadPoolExecutor(args.threads) as pool:
            c0 = os.times()
            t = time.perf_counter()
            total = sum(pool.map(host_write, range(n)))
            el = time.perf_counter() - t
            c1 = os.times()
        out["host_file_writes_only"] = {"GiBps": round(total / GIB / el, 3), "s": round(el, 4),
                                        "host_cores_busy": round((c1.user + c1.system - c0.user - c0.system) / el, 2)}
        list(ThreadPoolExecutor(args.threads).map(gpu_put, range(n)))  # restore the objects

        def ref_put(o):
            """filesystem.rs:686-828 with the crate algorithm (oracle/) and
            hashlib: write the data chunks, encode, write parity, manifest."""
            d = os.path.join(base, f"ref{o}.ec")
            os.makedirs(d, exist_ok=True)
            body = block[o % 4096: o % 4096 + size]
            chunks = [body[i * S:(i + 1) * S] for i in range(k)]
            dig = []
            for i, c in enumerate(chunks):  # write_chunk: file + Sha256 (SHA-NI via OpenSSL)
                with open(os.path.join(d, f"{i:06}"), "wb") as f:
                    f.write(c.tobytes())
                dig.append(hashlib.sha256(c).hexdigest())
            for i, p in enumerate(oracle.encode(chunks, m, S)):  # compute_and_write_parity
                with open(os.path.join(d, f"{k + i:06}"), "wb") as f:
                    f.write(p.tobytes())
                dig.append(hashlib.sha256(p).hexdigest())
            with open(os.path.join(d, "manifest.json"), "w") as f:
                json.dump({"chunks": dig}, f)
            return size

        for threads in (1, args.threads):
            t = time.perf_counter()
            with ThreadPoolExecutor(threads) as pool:
                total = sum(pool.map(ref_put, range(args.cpu_objects)))
            el = time.perf_counter() - t
            out[f"cpu_reference_put_{threads}t"] = {"GiBps": round(total / GIB / el, 3),
                                                   "objects": args.cpu_objects}
        lib = maxio_amd.lib()
        tls = threading.local()  # one output buffer per request thread

        def gpu_get(i_d):
            i, d = i_d
            b = getattr(tls, "buf", None)
            if b is None:
                b = tls.buf = ctx.host_array(size) if args.pinned else np.zeros(size, np.uint8)
            got = ctypes.c_uint64(0)
            rc = lib.mxec_get_object_chunked(ctx.handle, d.encode(), 0, (1 << 64) - 1,
                                             b.ctypes.data, size, ctypes.byref(got))
            assert rc == 0 and got.value == size, rc
            return got.value

        def timed(fn, items, threads):
            with ThreadPoolExecutor(threads) as pool:
                list(pool.map(fn, items[: threads]))  # warm
                best = None
                for _ in range(args.reps):
                    c0 = os.times()
                    t = time.perf_counter()
                    total = sum(pool.map(fn, items))
                    el = time.perf_counter() - t
                    c1 = os.times()
                    if best is None or el < best:
                        best = el
                        # host cores kept busy (user + system CPU time / wall)
                        cores[0] = round((c1.user + c1.system - c0.user - c0.system) / el, 2)
            return total / GIB / best, best

        cores = [None]

        items = list(enumerate(dirs))

        def host_read(i_d):
            """The file reads of a healthy GET alone (no hashing, no GPU):
            what the host side can deliver."""
            _, d = i_d
            total = 0
            for j in range(k):
                with open(os.path.join(d, f"{j:06}"), "rb") as f:
                    total += len(f.read())
            return total

        v, el = timed(host_read, items, args.threads)
        out["host_file_reads_only"] = {"GiBps": round(v, 3), "s": round(el, 4), "host_cores_busy": cores[0]}
        v, el = timed(gpu_get, items, args.threads)
        out["gpu_healthy"] = {"GiBps": round(v, 3), "s": round(el, 4), "host_cores_busy": cores[0]}
        one = items[:16]
        v1, el1 = timed(gpu_get, one, 1)
        # (round 1 divided by 16 whatever the object count: its 8-object
        # runs reported half the per-GET time)
        out["gpu_healthy_1thread"] = {"GiBps": round(v1, 3), "ms_per_object": round(el1 * 1e3 / len(one), 2)}
        # degraded: delete `erasures` data chunks of every object
        for o, d in enumerate(dirs):
            for i in np.random.default_rng(o).choice(k, args.erasures, replace=False):
                os.unlink(os.path.join(d, f"{int(i):06}"))
        v, el = timed(gpu_get, items, args.threads)
        out["gpu_degraded"] = {"GiBps": round(v, 3), "s": round(el, 4), "erasures_per_object": args.erasures,
                               "host_cores_busy": cores[0]}
        # bit-exactness of one degraded GET against the body written
        got = ctx.get_object_chunked(dirs[1])
        out["degraded_roundtrip_ok"] = got == block[1: 1 + size].tobytes()
        # the reference algorithm on the host cores (degraded objects)
        cpu_items = dirs[: args.cpu_objects]
        for threads in (1, args.threads):
            t = time.perf_counter()
            with ThreadPoolExecutor(threads) as pool:
                total = sum(pool.map(lambda d: reference_get(d, oracle), cpu_items))
            el = time.perf_counter() - t
            out[f"cpu_reference_degraded_{threads}t"] = {"GiBps": round(total / GIB / el, 3),
                                                         "objects": len(cpu_items)}
        ctx.close()
    finally:
        shutil.rmtree(base, ignore_errors=True)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
