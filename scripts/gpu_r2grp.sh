#!/bin/bash
# Grouped-launch geometry for config 5 (batch calls): V x workgroups per CU,
# alternating, two rounds; the mixed-batch tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/grp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mixed_batch_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for g in ${GEOMS:-4:32 2:32 4:16 2:64 4:48}; do
    V=${g%%:*}; B=${g##*:}
    MXEC_RS_GROUP_VECS=$V MXEC_RS_GROUP_BPC=$B timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-extra --cpu-seconds 0 > $O/cfg5_${V}_${B}_$r.json 2> $O/cfg5_${V}_${B}_$r.err || { tail -20 $O/cfg5_${V}_${B}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/cfg5_${V}_${B}_$r.json')); print('V=$V bpc=$B r$r', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['spot_check_vs_oracle'])"
  done
done
