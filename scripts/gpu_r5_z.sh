#!/bin/bash
# Round 5: the verified GET's uploads by SDMA against waves now that
# chain-bound waves ramp their pieces (128 / 256 / 512 objects).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5z}
mkdir -p $out
timeout -k 10 500 python -u tools/watch_diag.py --objects 128,256,512 --kinds verified,put_sha --modes auto,waves --reps 3 \
  > $out/verified_up.jsonl 2> $out/verified_up.err || { tail -5 $out/verified_up.err; exit 1; }
python3 -c "
import json
for l in open('$out/verified_up.jsonl'):
    r=json.loads(l); print(r['objects'], r['kind'], r['mode'], r['median_s'], [(c['s'], c['wave_blocks'], c['verify_groups']) for c in r['calls']])
"
