#!/bin/bash
# Round-2 evidence: the driver's default bench command, the same command
# under rocprofv3 --kernel-trace --stats, config 3c under a kernel trace, and
# a PMC VALU pass over the stream-form SHA kernel of config 3c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2n
mkdir -p $O
echo "== bench default"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']); print({k: d['extra'][k].get('roofline') for k in ('ns','config3','config3c')}); print(d['extra']['config3c']['GiBps_payload'], d['extra']['calibration'])"
cd /tmp && export TMPDIR=/tmp
echo "== rocprof default bench"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r2n_def -o run --output-format csv -- python3 "$R/bench.py" > "$R/$O/bench_rocprof.json" 2> "$R/$O/bench_rocprof.err" || { tail -5 "$R/$O/bench_rocprof.err"; exit 1; }
find /tmp/r2n_def -name "*kernel_stats.csv" -exec cp {} "$R/$O/default_kernel_stats.csv" \;
echo "== rocprof 3c"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r2n_3c -o run --output-format csv -- python3 "$R/bench.py" --config 3c --steps 6 --warmup 2 --cpu-seconds 0 > "$R/$O/cfg3c_rocprof.json" 2> "$R/$O/cfg3c_rocprof.err" || { tail -5 "$R/$O/cfg3c_rocprof.err"; exit 1; }
find /tmp/r2n_3c -name "*kernel_stats.csv" -exec cp {} "$R/$O/cfg3c_kernel_stats.csv" \;
find /tmp/r2n_3c -name "*kernel_trace.csv" -exec cp {} "$R/$O/cfg3c_kernel_trace.csv" \;
echo "== PMC VALU, stream SHA kernel (config 3c)"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex sha256_stream -d /tmp/r2n_pmc -o run --output-format csv -- python3 "$R/bench.py" --config 3c --steps 2 --warmup 1 --cpu-seconds 0 > "$R/$O/pmc_3c.log" 2>&1 || { tail -5 "$R/$O/pmc_3c.log"; exit 1; }
find /tmp/r2n_pmc -name "*counter_collection.csv" -exec cp {} "$R/$O/pmc_valu_3c.csv" \;
cd "$R"
ls -la $O
