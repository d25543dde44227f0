#!/bin/bash
# Replicated CRC tables: body-digest parity tests, then bench sums with the
# single-copy and replicated forms, two alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_digest_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MXEC_CRC_FORM=single timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_digest_gpu.py > $O/tests_single.log 2>&1 || { tail -30 $O/tests_single.log; exit 1; }
tail -1 $O/tests_single.log
for r in 1 2; do
 for f in single rep; do
  MXEC_CRC_FORM=$f timeout -k 10 400 python bench.py --config sums --steps 3 --warmup 1 --cpu-seconds 0 > $O/sums_${f}_$r.json 2> $O/sums_${f}_$r.err || { tail -20 $O/sums_${f}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/sums_${f}_$r.json')); r=d['roofline']; b=d['extra']['breakdown']; print('round $r $f', d['value'], r['achieved'], r['frac'], b['crc32c'], b['crc32'], d['spot_check_vs_oracle'])"
 done
done
