#!/bin/bash
# A/B of a library change on one box: bench configs (CONFIGS) with the
# library built from the previous kernel (build_ab/libmaxio_ec_prev.so, via
# MXEC_LIB) and with the current one, alternating, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/ab; mkdir -p $O
for r in ${ROUNDS:-1 2}; do
 for v in prev new; do
  if [ $v = prev ]; then export MXEC_LIB=$PWD/build_ab/libmaxio_ec_prev.so; else unset MXEC_LIB; fi
  for c in ${CONFIGS:-3c}; do
   timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/cfg${c}_$v$r.json 2> $O/cfg${c}_$v$r.err || { tail -20 $O/cfg${c}_$v$r.err; exit 1; }
   python -c "import json; d=json.load(open('$O/cfg${c}_$v$r.json')); print('$v cfg $c', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['spot_check_vs_oracle'], d.get('extra'))"
  done
 done
done
