#!/bin/bash
# Stream-form SHA-256 with one or two persistent waves per SIMD: its GPU
# tests, then config 3c alternating MXEC_SHA_STREAM_WPS (fresh process each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${1:?out subdir}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_sha_stream_gpu.py -x -v --timeout 250 --timeout-method thread \
  > "$O/pytest_stream.log" 2>&1 || { tail -40 "$O/pytest_stream.log"; exit 1; }
tail -1 "$O/pytest_stream.log"
for r in 1 2; do
  for w in 1 2; do
    MXEC_SHA_STREAM_WPS=$w timeout -k 10 300 python bench.py --config 3c --steps 8 --warmup 3 --cpu-seconds 0 --no-extra \
      > "$O/cfg3c_wps${w}_r$r.json" 2> "$O/cfg3c_wps${w}_r$r.err" || { tail -20 "$O/cfg3c_wps${w}_r$r.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('wps', sys.argv[2], d['value'], d['ms_per_step'], d['roofline'].get('frac'))" "$O/cfg3c_wps${w}_r$r.json" $w
  done
done
