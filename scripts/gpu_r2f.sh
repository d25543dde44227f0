#!/bin/bash
# Round 2: full -m gpu suite, SHA stream lab (big), configs 3c / 3, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2f; mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== lab big"; timeout -k 5 240 tools/sha_stream_lab big > $O/lab_big.jsonl 2>&1 || { cat $O/lab_big.jsonl; exit 1; }
cat $O/lab_big.jsonl
for c in "3c --workers 8" "3" "3c --workers 12" "3c --workers 4"; do
  tag=$(echo $c | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0 > $O/cfg$tag.json 2> $O/cfg$tag.err || { tail -20 $O/cfg$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg$tag.json')); print('$c', d['value'], d['ms_per_step'], d['spot_check_vs_oracle'], d.get('extra'))"
done
echo "== bench default"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline'].get('frac_of_box_stream')); e=d['extra']; print({k: e[k].get('roofline') for k in ('ns','config3','config3c')}); print(e['config3c']['GiBps_payload'], e['calibration'])"
