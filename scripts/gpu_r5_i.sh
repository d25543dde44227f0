#!/bin/bash
# Round 5: where a GET's extra time goes after 60 GB of HBM is freed --
# the lab build's per-wave pipeline trace (copy / decode / download events),
# fresh and after the free, SDMA and waves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5i}
mkdir -p $out
export MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_PIPE_TRACE=1
timeout -k 10 300 python -u tools/watch_diag.py --objects 128 --kinds rs,verified --modes sdma,waves --reps 3 \
  > $out/trace_fresh.jsonl 2> $out/trace_fresh.err || { tail -5 $out/trace_fresh.err; exit 1; }
timeout -k 10 300 python -u tools/watch_diag.py --objects 128 --kinds rs,verified --modes sdma,waves --reps 3 --churn-each 60 \
  > $out/trace_churn.jsonl 2> $out/trace_churn.err || { tail -5 $out/trace_churn.err; exit 1; }
for f in trace_fresh trace_churn; do python3 -c "
import json
for l in open('$out/$f.jsonl'):
    r=json.loads(l); print('$f', r['kind'], r['mode'], r.get('free_s'), [c['s'] for c in r['calls']])
"; done
