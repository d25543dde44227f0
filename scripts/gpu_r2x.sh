#!/bin/bash
# Hash-wave priority (MXEC_SHA_PRIO 0 / 3) now that the speculative decodes
# run beside the combined hash: config 3c and config 3, two alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2x2; mkdir -p $O
for r in 1 2; do
 for p in 0 3; do
  MXEC_SHA_PRIO=$p timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 8 --warmup 2 --cpu-seconds 0 > $O/cfg3c_p${p}_$r.json 2> $O/cfg3c_p${p}_$r.err || { tail -20 $O/cfg3c_p${p}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3c_p${p}_$r.json')); r=d['roofline']; print('round $r prio $p 3c', d['value'], d['ms_per_step'])"
  MXEC_SHA_PRIO=$p timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg3_p${p}_$r.json 2> $O/cfg3_p${p}_$r.err || { tail -20 $O/cfg3_p${p}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_p${p}_$r.json')); print('round $r prio $p 3', d['value'], d['ms_per_step'])"
 done
done
