#!/bin/bash
# Round 5: does freeing HBM slow the SDMA copies right after (the kernel
# driver wiping released VRAM)?  60 GB freed between each warm call and its
# timed calls, SDMA against waves; then (last: may fault at exit) the
# torch-only eight-stream exit probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5h}
mkdir -p $out
timeout -k 10 400 python -u tools/watch_diag.py --objects 128 --kinds verified,rs,put_rs --modes sdma,waves,auto --reps 6 --churn-each 60 \
  > $out/engine_churn_each.jsonl 2> $out/engine_churn_each.err || { tail -5 $out/engine_churn_each.err; exit 1; }
python3 -c "
import json
for l in open('$out/engine_churn_each.jsonl'):
    r=json.loads(l); print(r['objects'], r['kind'], r['mode'], r.get('free_s'), [c['s'] for c in r['calls']], [c['sdma_slow'] for c in r['calls']], [c['sdma_last_mbps'] for c in r['calls']])
"
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_s -o run --output-format csv \
  -- python3 $R/tools/exit_probe.py torch_streams > $R/$out/exit_torch_streams.out 2> $R/$out/exit_torch_streams.err
echo "{\"what\": \"torch_streams (eight streams, torch only)\", \"rc\": $?}" | tee -a $R/$out/exit_probe5.jsonl
