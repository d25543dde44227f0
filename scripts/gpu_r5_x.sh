#!/bin/bash
# Round 5: why the default line's PUT with digests got a slow verdict with
# the piece ramp: per-piece upload marks (lab MXEC_PIPE_TRACE) fresh and
# after a 74 GB free, watch counters per call; then config 3 without the
# K + W ring's barriers (make nosync) against the lab build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5x}
mkdir -p $out
export MXEC_PIPE_TRACE=1
for c in 0 74; do
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so timeout -k 10 300 python -u tools/watch_diag.py --objects 128 --kinds put_rs,put_sha --modes auto --reps 3 --churn $c \
  > $out/putsha_churn$c.jsonl 2> $out/putsha_churn$c.err || { tail -5 $out/putsha_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/putsha_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['kind'], r['median_s'], [(c['s'], c['sdma_checks'], c['sdma_slow'], c['sdma_last_mbps'], c['wave_blocks']) for c in r['calls']])
"
done
unset MXEC_PIPE_TRACE
for lib in lab lab_nosync; do
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_$lib.so timeout -k 10 300 python bench.py --config 3 --no-extra --no-e2e --cpu-seconds 0 --steps 10 --warmup 3 \
  > $out/cfg3_$lib.json 2> $out/cfg3_$lib.err || { tail -5 $out/cfg3_$lib.err; exit 1; }
python3 -c "
import json;d=json.load(open('$out/cfg3_$lib.json'));print('$lib', d['value'], d['ms_per_step'], d['roofline'].get('ms_per_launch'))"
done
