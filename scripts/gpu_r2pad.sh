#!/bin/bash
# Shard-slot padding A/B on whatever box this is: pad 0 vs 2 MiB + 64 KiB,
# alternating processes, 12 re-allocations each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2pad_$(date +%s); mkdir -p $O
for rep in 1 2; do
for pad in 0 2162688; do
  timeout -k 10 400 python tools/alloc_lab.py --allocs 12 --reps 3 --alloc torch --layout object_major --pad $pad > $O/pad_${pad}_$rep.jsonl 2> $O/pad_${pad}_$rep.err || { tail -20 $O/pad_${pad}_$rep.err; exit 1; }
  python -c "
import json
v=[json.loads(l)['rs_TBps'] for l in open('$O/pad_${pad}_$rep.jsonl')]
print('rep $rep pad $pad min %.3f mean %.3f max %.3f' % (min(v), sum(v)/len(v), max(v)), v)"
done
done
