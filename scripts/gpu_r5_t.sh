#!/bin/bash
# Round 5: where the 512-object verified GET's time goes at two
# verification groups (lab build, MXEC_PIPE_TRACE=1), and the bench default
# line at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5t}
mkdir -p $out
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_PIPE_TRACE=1 timeout -k 10 300 python -u tools/watch_diag.py --objects 512 --kinds verified --modes auto --reps 2 \
  > $out/trace512.jsonl 2> $out/trace512.err || { tail -5 $out/trace512.err; exit 1; }
cat $out/trace512.jsonl
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/bench.json'));print(d['value'],d['roofline']['frac']);e=d['extra']
for k in ('e2e_host','e2e_get_after_extras'):
  for kk,vv in e[k].items():
    if isinstance(vv,dict) and 's_each' in vv: print(k,kk,vv['s_each'])
"
