#!/bin/bash
# Stream form with 1 vs 4 waves per workgroup (check + timing at 20k-131k
# messages), then config 3c with the combiner log (device-side event hand-off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2g; mkdir -p $O
timeout -k 5 120 tools/sha_stream_lab check > $O/lab_check.jsonl 2>&1 || { cat $O/lab_check.jsonl; exit 1; }
grep wg4 $O/lab_check.jsonl
timeout -k 5 300 tools/sha_stream_lab big > $O/lab_big.jsonl 2>&1 || { cat $O/lab_big.jsonl; exit 1; }
cat $O/lab_big.jsonl
MXEC_COMBINE_LOG=1 timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 6 --warmup 2 --cpu-seconds 0 > $O/cfg3c.json 2> $O/cfg3c.err || { tail -20 $O/cfg3c.err; exit 1; }
grep "mxec combine" $O/cfg3c.err | tail -12
python -c "import json; d=json.load(open('$O/cfg3c.json')); print(d['value'], d['ms_per_step'], d['extra'])"
