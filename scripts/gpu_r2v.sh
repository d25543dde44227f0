#!/bin/bash
# Tile interleave across objects (MXEC_RS_INTERLEAVE) on the same
# allocations; parity of the interleaved order first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2v; mkdir -p $O
MXEC_RS_INTERLEAVE=7 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_configs_gpu.py > $O/tests_ilv.log 2>&1 || { tail -30 $O/tests_ilv.log; exit 1; }
tail -1 $O/tests_ilv.log
timeout -k 10 400 python tools/alloc_lab.py --allocs 8 --reps 5 --alloc torch > $O/alloc_ilv.jsonl 2> $O/alloc_ilv.err || { tail -20 $O/alloc_ilv.err; exit 1; }
python -c "
import json
for l in open('$O/alloc_ilv.jsonl'):
    d = json.loads(l); print(d['alloc'], d['rs_TBps'], d['rs_ilv8_TBps'], d['rs_ilv32_TBps'], d['rs_ilv256_TBps'], 'pattern', d['pattern_TBps'], 'wr', d['write_parity_nt_TBps'])"
