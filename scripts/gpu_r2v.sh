#!/bin/bash
# Allocation spread by layout: data then parity (the bench), parity first,
# one object-major [n][k+m][S] tensor; 8 re-allocations each, one process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2v; mkdir -p $O
for lay in separate object_major parity_first object_major separate; do
  timeout -k 10 400 python tools/alloc_lab.py --allocs 8 --reps 3 --alloc torch --layout $lay > $O/lay_$lay.jsonl 2> $O/lay_$lay.err || { tail -20 $O/lay_$lay.err; exit 1; }
  python -c "
import json
print('$lay', [json.loads(l)['rs_TBps'] for l in open('$O/lay_$lay.jsonl')])"
done
