#!/bin/bash
# Round 2, RS VALU change: -m gpu suite on the new library, then an A/B of
# the RS kernel (build_ab/libmaxio_ec_prev.so = previous rs_kernel.hip,
# everything else identical) on configs 2 / ns / 4a / 5 / 3, alternating
# prev/new twice on one box, PMC VALU counters for the new R=4 kernel, and
# the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2b
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== A/B"
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export MXEC_LIB=$R/build_ab/libmaxio_ec_prev.so; else unset MXEC_LIB; fi
    for c in ${CONFIGS:-2 ns 4a 5 3}; do
      timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-extra > $O/cfg${c}_$v$r.json 2> $O/cfg${c}_$v$r.err || { tail -20 $O/cfg${c}_$v$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/cfg${c}_$v$r.json')); r=d['roofline']; print('$v$r cfg $c', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream_GBps'), r.get('frac_of_box_stream'), d['spot_check_vs_oracle'])"
    done
  done
done
unset MXEC_LIB
cd /tmp && export TMPDIR=/tmp
echo "== PMC VALU, new kernel, config ns and 2 (no extras)"
for cfg in ns 2; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex rs_apply_fast -d "/tmp/pmcb_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --cpu-seconds 0 --no-extra > "$R/$O/pmc_$cfg.log" 2>&1 || { tail -5 "$R/$O/pmc_$cfg.log"; exit 1; }
  find "/tmp/pmcb_$cfg" -name "*counter_collection.csv" -exec cp {} "$R/$O/pmc_valu_$cfg.csv" \;
done
cd "$R"
echo "== bench default"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']); print(d['extra']['calibration']); print({k: d['extra'][k].get('roofline') for k in ('ns','config3','config3c')})"
