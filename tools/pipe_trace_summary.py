#!/usr/bin/env python3
"""Summarise tools/pipe_trace.py's stderr (MXEC_PIPE_TRACE wave lines,
pipeline.cpp PipeTrace): per phase and wave, the GPU marks by kind (first /
last time, count) and the host marks, all in ms against one reference.

  python tools/pipe_trace_summary.py gpurun_out/r6d/trace_auto.err
"""
from __future__ import annotations

import collections
import json
import sys


def main() -> int:
    phase = None
    for line in open(sys.argv[1]):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "phase_start" in d:
            phase = d["phase_start"]
            print(f"== {phase}")
            continue
        if "pipe_trace" not in d:
            continue
        by = collections.OrderedDict()
        for name, ms in d["gpu_ms"]:
            by.setdefault(name, []).append(ms)
        t0 = min(ms for _, ms in d["gpu_ms"]) if d["gpu_ms"] else 0
        gpu = "  ".join(f"{n}[{len(v)}] {min(v):.1f}-{max(v):.1f}" for n, v in by.items())
        hb = collections.OrderedDict()
        for name, ms in d["host_ms"]:
            hb.setdefault(name, []).append(ms)
        host = "  ".join(f"{n}[{len(v)}] {min(v):.1f}-{max(v):.1f}" for n, v in hb.items())
        print(f"  {d['pipe_trace']}: gpu {gpu}\n      host {host}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
