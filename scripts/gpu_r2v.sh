#!/bin/bash
# Config-2 spread by allocation: RS kernel vs the probe streams on the SAME
# buffers, six re-allocations in one process (torch allocator).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2v; mkdir -p $O
timeout -k 10 400 python tools/alloc_lab.py --allocs 8 --reps 5 --alloc torch > $O/alloc_probe.jsonl 2> $O/alloc_probe.err || { tail -20 $O/alloc_probe.err; exit 1; }
cut -c1-300 $O/alloc_probe.jsonl
