#!/bin/bash
# Round 2: -m gpu suite, then a three-way A/B of the RS kernel on one box
# (prev = round-1 kernel, pairall = paired MAC at every R, cur = paired MAC
# for R >= 3 only), interleaved, ROUNDS rounds, configs 2 / ns / 4a / 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2c
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in prev pairall cur; do
    case $v in
      prev) export MXEC_LIB=$R/build_ab/libmaxio_ec_prev.so ;;
      pairall) export MXEC_LIB=$R/build_ab/libmaxio_ec_pairall.so ;;
      cur) unset MXEC_LIB ;;
    esac
    for c in ${CONFIGS:-2 ns 4a 5}; do
      timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-extra > $O/cfg${c}_$v$r.json 2> $O/cfg${c}_$v$r.err || { tail -20 $O/cfg${c}_$v$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/cfg${c}_$v$r.json')); r=d['roofline']; print('$v$r cfg $c', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream_GBps'), r.get('frac_of_box_stream'), d['spot_check_vs_oracle'])"
    done
  done
done
