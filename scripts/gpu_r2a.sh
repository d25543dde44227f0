#!/bin/bash
# Round 2, first GPU call: the -m gpu suite (with the new multi-device and
# pinned error-path tests), the default bench line (headline + extras), the
# chip-wide VALU issue lab, rocprofv3 kernel stats of the default bench, and
# PMC VALU / occupancy counters for the R=2 vs R=4 RS kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2a
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== valu_lab chip"
timeout -k 10 120 tools/valu_lab chip > $O/valu_chip.jsonl 2>&1 || { cat $O/valu_chip.jsonl; exit 1; }
cat $O/valu_chip.jsonl
echo "== bench (default)"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
echo "== rocprofv3 kernel stats (default bench, no CPU leg)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --cpu-seconds 0 > "$R/$O/prof_bench.json" 2> "$R/$O/prof_bench.err" || { tail "$R/$O/prof_bench.err"; exit 1; }
find "$R/$O/prof" -name "*kernel_stats.csv" -exec cp {} "$R/$O/kernel_stats.csv" \;
head -12 "$R/$O/kernel_stats.csv"
echo "== PMC: VALU / busy / waves per RS kernel (configs 2, ns)"
for cfg in 2 ns; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex rs_apply_fast -d "/tmp/pmc_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --cpu-seconds 0 > "$R/$O/pmc_$cfg.log" 2>&1 || { tail -5 "$R/$O/pmc_$cfg.log"; exit 1; }
  find "/tmp/pmc_$cfg" -name "*counter_collection.csv" -exec cp {} "$R/$O/pmc_valu_$cfg.csv" \;
done
echo "== PMC: SHA kernel VALU (config 3)"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex sha256 -d "/tmp/pmc_3" -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 2 --warmup 1 --cpu-seconds 0 > "$R/$O/pmc_3.log" 2>&1 || { tail -5 "$R/$O/pmc_3.log"; exit 1; }
find "/tmp/pmc_3" -name "*counter_collection.csv" -exec cp {} "$R/$O/pmc_valu_3.csv" \;
ls -la "$R/$O"
