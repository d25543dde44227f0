#!/bin/bash
# Round 5: a piece ramp for the grouped verified GET (lab MXEC_PIPE_RAMP_KB):
# a group's verdict comes one chain after its FIRST piece is up, so a small
# first piece should pull every verdict earlier.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5u}
mkdir -p $out
export MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for r in 0 256 1024; do
MXEC_PIPE_RAMP_KB=$r timeout -k 10 300 python -u tools/watch_diag.py --objects 128,512 --kinds verified,put_sha --modes auto --reps 3 \
  > $out/ramp_$r.jsonl 2> $out/ramp_$r.err || { tail -5 $out/ramp_$r.err; exit 1; }
python3 -c "
import json
for l in open('$out/ramp_$r.jsonl'):
    r=json.loads(l); print('ramp $r', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']])
"
done
