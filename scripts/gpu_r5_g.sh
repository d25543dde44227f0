#!/bin/bash
# Round 5: copy engine by measurement -- SDMA against CU waves for every
# host batch kind at 128 and 512 objects, in a fresh process and after 74 GB
# of HBM churn (bench.py's headline allocation).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5g}
mkdir -p $out
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds verified,rs,put_rs,put_sha --modes sdma,waves \
  > $out/engine_fresh.jsonl 2> $out/engine_fresh.err || { tail -5 $out/engine_fresh.err; exit 1; }
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds verified,rs,put_rs,put_sha --modes auto,sdma,waves --churn 74 \
  > $out/engine_churn.jsonl 2> $out/engine_churn.err || { tail -5 $out/engine_churn.err; exit 1; }
python3 -c "
import json
for f in ('engine_fresh','engine_churn'):
    for l in open('$out/'+f+'.jsonl'):
        r=json.loads(l); print(f, r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']], sum(c['sdma_slow'] for c in r['calls']))
"
# Last (it may fault at exit): does torch's own async copy arm the
# profiler's exit-time fault?
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_t -o run --output-format csv \
  -- python3 $R/tools/exit_probe.py torch_copy > $R/$out/exit_torch_copy.out 2> $R/$out/exit_torch_copy.err
echo "{\"what\": \"torch_copy (no mxec call but open)\", \"rc\": $?}" | tee -a $R/$out/exit_probe4.jsonl
