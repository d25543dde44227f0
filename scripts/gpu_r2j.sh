#!/bin/bash
# Full GPU suite, config 3c (new step roofline) and the lab at the form
# crossover sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MXEC_COMBINE_LOG=1 timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 8 --warmup 2 --cpu-seconds 0 > $O/cfg3c.json 2> $O/cfg3c.err || { tail -20 $O/cfg3c.err; exit 1; }
grep "mxec combine" $O/cfg3c.err | tail -4
python -c "import json; d=json.load(open('$O/cfg3c.json')); print(d['value'], d['ms_per_step'], d.get('roofline'))"
LAB_SIZES=45056,49152,53248,57344 timeout -k 5 200 tools/sha_stream_lab big > $O/lab_sizes.jsonl 2>&1 || { cat $O/lab_sizes.jsonl; exit 1; }
cat $O/lab_sizes.jsonl
