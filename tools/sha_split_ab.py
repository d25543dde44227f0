#!/usr/bin/env python3
"""Within-process A/B of the SHA-256 split form (config 3's verify launch:
10 240 x 1 MiB messages) over a knob read per launch, alternating rounds,
HIP-event timed; digests compared across arms and against hashlib for a
sample.  Lab tool, not product.

  python tools/sha_split_ab.py [--env MXEC_SHA_SPLIT_BUFS] [--values 3,2]
      [--messages 10240] [--size 1048576] [--rounds 3] [--reps 3]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# The lab knobs exist only in the lab build (make -C maxio_amd/csrc lab).
os.environ.setdefault("MXEC_LIB", os.path.join(ROOT, "maxio_amd", "lib", "libmaxio_ec_lab.so"))

import bench  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="MXEC_SHA_SPLIT_BUFS")
    ap.add_argument("--values", default="3,2")
    ap.add_argument("--messages", type=int, default=10240)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import maxio_amd

    dev = torch.device("cuda", 0)
    ctx = maxio_amd.Context(device_mask=1, streams_per_device=2)
    st = torch.cuda.Stream(device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    buf = torch.randint(0, 256, (a.messages, a.size), dtype=torch.uint8, device=dev, generator=g)
    ptrs = [buf[i].data_ptr() for i in range(a.messages)]
    lens = [a.size] * a.messages
    dig = torch.empty((a.messages, 32), dtype=torch.uint8, device=dev)
    seen = {}
    for rnd in range(a.rounds):
        for val in a.values.split(","):
            if val:
                os.environ[a.env] = val
            else:
                os.environ.pop(a.env, None)
            ms = bench.event_ms(torch, st, lambda: ctx.sha256_batch_device(ptrs, lens, dig.data_ptr(),
                                                                           stream=st.cuda_stream), a.reps)
            torch.cuda.synchronize()
            d = dig.cpu().numpy().copy()
            if val in seen:
                assert (seen[val] == d).all()
            seen[val] = d
            print(json.dumps({"round": rnd, a.env: val, "ms": round(ms, 4),
                              "us_per_block": round(ms * 1e3 / (a.size / 64), 4)}), flush=True)
    os.environ.pop(a.env, None)
    arms = list(seen.values())
    same = all((x == arms[0]).all() for x in arms)
    sample = [0, a.messages // 2, a.messages - 1]
    ok = all(hashlib.sha256(buf[i].cpu().numpy().tobytes()).digest() == arms[0][i].tobytes() for i in sample)
    print(json.dumps({"digests_equal_across_arms": bool(same), "hashlib_sample_ok": bool(ok)}), flush=True)
    ctx.close()
    return 0 if same and ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
