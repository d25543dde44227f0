#!/bin/bash
# Padded shard strides, more samples: 12 re-allocations, two processes per pad.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2v2; mkdir -p $O
for rep in 1 2; do
for pad in 0 1048576 1052672 2162688 3145728; do
  timeout -k 10 400 python tools/alloc_lab.py --allocs 12 --reps 3 --alloc torch --layout object_major --pad $pad > $O/pad_${pad}_$rep.jsonl 2> $O/pad_${pad}_$rep.err || { tail -20 $O/pad_${pad}_$rep.err; exit 1; }
  python -c "
import json
v=[json.loads(l)['rs_TBps'] for l in open('$O/pad_${pad}_$rep.jsonl')]
print('rep $rep pad $pad min %.3f mean %.3f max %.3f' % (min(v), sum(v)/len(v), max(v)), v)"
done
done
