#!/bin/bash
# Round 5: the piece ramp A/B at the final copy policy (lab override
# MXEC_PIPE_RAMP_KB=0 against the default 256 KiB ramp of chain-bound waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5ab}
mkdir -p $out
export MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for r in 0 256 0 256; do
MXEC_PIPE_RAMP_KB=$r timeout -k 10 300 python -u tools/watch_diag.py --objects 128 --kinds verified,put_sha --modes auto --reps 5 \
  >> $out/ramp_ab.jsonl 2>> $out/ramp_ab.err || { tail -5 $out/ramp_ab.err; exit 1; }
done
python3 -c "
import json
for i,l in enumerate(open('$out/ramp_ab.jsonl')):
    r=json.loads(l); print(['ramp0','ramp256'][(i//2)%2], r['kind'], r['median_s'], [c['s'] for c in r['calls']])
"
