#!/bin/bash
# Round 5: verification groups again, now that the verified GET's downloads
# go by waves (does the download overlap the later groups' uploads now?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5r}
mkdir -p $out
for g in 1 2 3 4; do
MXEC_GET_VGROUPS=$g timeout -k 10 300 python -u tools/watch_diag.py --objects 512 --kinds verified --modes auto,sdma --reps 3 \
  > $out/vgroups_$g.jsonl 2> $out/vgroups_$g.err || { tail -5 $out/vgroups_$g.err; exit 1; }
python3 -c "
import json
for l in open('$out/vgroups_$g.jsonl'):
    r=json.loads(l); print('G=$g', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']])
"
done
