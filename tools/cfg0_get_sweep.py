#!/usr/bin/env python3
"""configs[0]'s GET (k = 1, m = 2, 10 MiB chunks, one erasure) from page-cached
shard files at 1, 16 and 128 concurrent requests (tools/e2e_get_bench.py),
and the one-request stage latencies (tools/get_latency.py), each in a child
process; one JSON line per run (INTEGRATION.md "When a lone request is
slower on the GPU").  The parent never touches the GPU.

  python tools/cfg0_get_sweep.py --threads 1,16,128
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,16,128")
    a = ap.parse_args()
    runs = [(f"get_w{w}", ["e2e_get_bench.py", "--k", "1", "--parity", "2", "--chunk-size", "10485760",
                           "--erasures", "1", "--threads", w, "--objects", str(max(int(w), 8)), "--cpu-objects", "8"])
            for w in a.threads.split(",")] + [("latency", ["get_latency.py"])]
    for name, cmd in runs:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", cmd[0])] + cmd[1:], capture_output=True,
                             text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:], file=sys.stderr)
            return out.returncode
        for line in out.stdout.strip().splitlines():
            if line.startswith("{"):
                print(json.dumps({"run": name, **json.loads(line)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
