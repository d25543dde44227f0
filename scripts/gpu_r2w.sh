#!/bin/bash
# Speculative rebuild beside the combined hash: full GPU suite, then config
# 3c and the default bench (config 3 / 3c extras).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
MXEC_COMBINE_LOG=1 timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 8 --warmup 2 --cpu-seconds 0 > $O/cfg3c_$r.json 2> $O/cfg3c_$r.err || { tail -20 $O/cfg3c_$r.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3c_$r.json')); r=d['roofline']; print('3c', d['value'], d['ms_per_step'], r['frac'], r['frac_hash_only'])"
done
timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg3.json 2> $O/cfg3.err || { tail -20 $O/cfg3.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3.json')); print('3', d['value'], d['ms_per_step'], d['spot_check_vs_oracle'])"
LAB_SIZES=10240,81920 timeout -k 5 120 tools/sha_stream_lab big > $O/lab.jsonl 2>&1 || { cat $O/lab.jsonl; exit 1; }
cat $O/lab.jsonl
grep "mxec combine" $O/cfg3c_2.err | tail -4
