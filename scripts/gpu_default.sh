#!/bin/bash
# The driver's default bench command once, with a one-screen summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/default; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d["extra"]; r = d["roofline"]
print("headline", d["value"], d["ms_per_step"], r["frac"], r.get("frac_of_box_stream"))
print("ns", e["ns"]["GiBps_payload"], e["ns"]["roofline"]["frac"], e["ns"]["roofline"].get("frac_of_box_stream"))
print("3", e["config3"]["GiBps_payload"], e["config3"]["ms_per_call"], e["config3"]["rs_decode"])
print("5", e["config5"]["GiBps_payload"], e["config5"]["ms_per_step"], e["config5"]["roofline"])
print("3c", e["config3c"]["GiBps_payload"], e["config3c"]["roofline"]["frac"])
PY
