#!/bin/bash
# ns (800 KB descriptor tables per call) with the tables copied in the launch
# stream vs on the side stream: kernel trace gaps between launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); O=$R/gpurun_out/upl2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for up in inline stream; do
  MXEC_DESC_UPLOAD=$up timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$up -o run --output-format csv -- python3 $R/bench.py --config ns --steps 20 --warmup 2 --no-extra --cpu-seconds 0 > $O/ns_$up.json 2> $O/ns_$up.err || { tail -5 $O/ns_$up.err; exit 1; }
done
cd $R
for up in inline stream; do
python3 - $O/prof_$up $O/ns_$up.json <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "rs_apply_fast<4, 4, true, false" in r["Kernel_Name"]]
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ks, ks[1:])]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
d = json.load(open(sys.argv[2]))
print(sys.argv[1].split("_")[-1], "value", d["value"], "ms/step", d["ms_per_step"], "kernel avg us", round(sum(dur[3:]) / len(dur[3:]), 1), "gaps us", sorted(round(g, 1) for g in gaps[3:])[len(gaps[3:]) // 2])
PY
done
