#!/bin/bash
# Ch as one v_bitop3 (1541 -> 1415 VALU per block): hash parity tests, lab
# timings, config 3c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "sha or hash or digest or sums or stream or reconstruct or verify" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 5 120 tools/sha_stream_lab check > $O/lab_check.jsonl 2>&1 || { cat $O/lab_check.jsonl; exit 1; }
LAB_SIZES=10240,40960,49152,53248,81920 timeout -k 5 200 tools/sha_stream_lab big > $O/lab_big.jsonl 2>&1 || { cat $O/lab_big.jsonl; exit 1; }
cat $O/lab_big.jsonl
MXEC_COMBINE_LOG=1 timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 8 --warmup 2 --cpu-seconds 0 > $O/cfg3c.json 2> $O/cfg3c.err || { tail -20 $O/cfg3c.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3c.json')); print(d['value'], d['ms_per_step'], d.get('roofline'))"
