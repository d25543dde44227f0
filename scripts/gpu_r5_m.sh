#!/bin/bash
# Round 5: what the watch's brackets cost (auto vs auto with the watch off
# vs sdma), fresh; then how long a 60 GB free slows the GET (60 RS-only GETs
# by SDMA after one free).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5m}
mkdir -p $out
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds put_sha,rs,verified,put_rs --modes auto,auto_nowatch,sdma --reps 3 \
  > $out/watch_cost.jsonl 2> $out/watch_cost.err || { tail -5 $out/watch_cost.err; exit 1; }
python3 -c "
import json
for l in open('$out/watch_cost.jsonl'):
    r=json.loads(l); print(r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']], [(c.get('sdma_slow'), c.get('sdma_down_slow'), c.get('sdma_down_last_mbps')) for c in r['calls']])
"
timeout -k 10 200 python -u tools/watch_diag.py --objects 128 --kinds rs --modes sdma,waves --reps 60 --churn-each 60 \
  > $out/duration.jsonl 2> $out/duration.err || { tail -5 $out/duration.err; exit 1; }
python3 -c "
import json
for l in open('$out/duration.jsonl'):
    r=json.loads(l); print(r['kind'], r['mode'], [c['s'] for c in r['calls']])
"
