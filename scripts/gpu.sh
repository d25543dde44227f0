#!/bin/bash
# One parametrised GPU-box script (replaces round 2's one-off lease scripts).
#
#   scripts/gpu.sh <out-subdir> step[,step...]
#
# Steps (each under its own time limit; the first failure ends the call):
#   tests     full `pytest -m gpu` (one process) -> pytest_gpu.log
#   smoke     __graft_entry__.smoke()
#   bench     the driver's command: python bench.py (defaults --gpus 1 --steps 20
#             --warmup 5) -> bench.json
#   refuse2   python bench.py --gpus 2 on a one-GPU box: must exit 2, no line
#   rehearse  BENCH_REHEARSE_LOGICAL=1 bench.py --gpus 2 (labelled in-process
#             multi-device rehearsal on two logical devices of the one card)
#   rehearse8 the same with --gpus 8 on eight logical devices (64 objects each)
#   ranks2    the torch.distributed.run path with two ranks on the one GPU
#             (BENCH_GPU_OF_RANK=0, gloo for the timing collectives)
#   prof      rocprofv3 --kernel-trace --stats of the default bench command
#   trace     rocprofv3 --kernel-trace --memory-copy-trace of the default bench
#             with BENCH_GET_STAMPS=1 and BENCH_DUMP_MAPS=1 (the DSO map on
#             stderr before teardown); tools/get_trace_summary.py lines the
#             timed GET batches up with the trace -> get_trace_summary.json
#   pmc       FETCH_SIZE / WRITE_SIZE passes (one run each) of rs_apply_fast
#             for configs 2 and ns at every grid the tuner can pick (2: 1024 /
#             512 / 256, ns: 512 / 256 / 128), summarised with the grid (the
#             grid fixed through the lab build's MXEC_RS_BPC: make lab first)
#   clock     GRBM_GUI_ACTIVE / GRBM_COUNT pass (one run per config) of configs
#             3 (SHA-256 split form + decode) and 2 / ns (RS encode):
#             effective clock per kernel (tools/clock_summary.py)
#   rust      probe for rustc / cargo
#   cfg:<c>   python bench.py --config <c> --no-extra -> cfg_<c>.json
#   pmc5      FETCH_SIZE / WRITE_SIZE passes over config 5's step (grouped /
#             multi-r RS launches) -> r6_pmc_cfg5_grouped_traffic.json
#   exitprobe tools/exit_probe.py host_pageable under rocprofv3 --kernel-trace
#             --memory-copy-trace (the round-5 exit fault); last in a call
#   pyt:<f+f> the named test files only (tests/<f>.py, `+`-separated), -m gpu
#             -> pytest_<first>.log
#   tool:<t>  python tools/<t>.py $TOOL_ARGS_<t> (else $TOOL_ARGS) -> <t>.jsonl
#             (stderr <t>.err);
#             the round-4/5 study scripts' one-off runs (watch_diag,
#             sha_alone, exit_probe, concurrent_e2e, ...) go through this
# Env: BENCH_ARGS (extra bench.py args for bench/prof), TOOL_ARGS, TOOL_TIMEOUT
# (seconds, default 600).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O="$R/gpurun_out/${1:?out subdir}"
mkdir -p "$O"
IFS=, read -ra STEPS <<< "${2:?steps}"
export TMPDIR=/tmp
for st in "${STEPS[@]}"; do
  echo "== $st $(date +%T)"
  case "$st" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
      tail -2 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
      cat "$O/smoke.log" ;;
    bench)
      timeout -k 10 900 python bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
      cat "$O/bench.json" ;;
    refuse2)
      rc=0; timeout -k 10 300 python bench.py --gpus 2 --steps 2 > "$O/refuse2.out" 2> "$O/refuse2.err" || rc=$?
      echo "exit $rc"; cat "$O/refuse2.err"
      [ "$rc" = 2 ] && [ ! -s "$O/refuse2.out" ] || { echo "expected exit 2 and no line"; exit 1; } ;;
    rehearse)
      BENCH_REHEARSE_LOGICAL=1 timeout -k 10 600 python bench.py --gpus 2 --objects 256 --steps 10 --warmup 2 \
        > "$O/rehearse2.json" 2> "$O/rehearse2.err" || { tail -20 "$O/rehearse2.err"; exit 1; }
      cat "$O/rehearse2.json" ;;
    rehearse8)
      BENCH_REHEARSE_LOGICAL=1 timeout -k 10 600 python bench.py --gpus 8 --objects 64 --steps 10 --warmup 2 \
        > "$O/rehearse8.json" 2> "$O/rehearse8.err" || { tail -20 "$O/rehearse8.err"; exit 1; }
      cat "$O/rehearse8.json" ;;
    ranks2)
      BENCH_GPU_OF_RANK=0 BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --objects 256 --steps 10 \
        --warmup 2 > "$O/ranks2.json" 2> "$O/ranks2.err" || { tail -20 "$O/ranks2.err"; exit 1; }
      cat "$O/ranks2.json" ;;
    prof)
      ( cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv \
          -- python3 "$R/bench.py" $BENCH_ARGS > "$O/prof_bench.json" 2> "$O/prof_bench.err" ) || { tail -20 "$O/prof_bench.err"; exit 1; }
      find /tmp/prof -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
      find /tmp/prof -name "*kernel_trace.csv" -exec cp {} "$O/kernel_trace.csv" \;
      python tools/headline_timed.py "$O/kernel_trace.csv" "$O/prof_bench.json" --out "$O/headline_timed.json" || exit 1
      gzip -f "$O/kernel_trace.csv"
      cat "$O/prof_bench.json" ;;
    trace)
      ( cd /tmp && BENCH_GET_STAMPS=1 BENCH_DUMP_MAPS=1 timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/trace \
          -o run --output-format csv -- python3 "$R/bench.py" $BENCH_ARGS > "$O/trace_bench.json" \
          2> "$O/trace_bench.err" ) || { tail -20 "$O/trace_bench.err"; exit 1; }
      kt=$(find /tmp/trace -name "*kernel_trace.csv" -print -quit); mt=$(find /tmp/trace -name "*memory_copy_trace.csv" -print -quit)
      python tools/get_trace_summary.py "$kt" "$mt" "$O/trace_bench.json" --out "$O/get_trace_summary.json" > /dev/null \
        || exit 1
      gzip -c "$kt" > "$O/kernel_trace.csv.gz"; gzip -c "$mt" > "$O/memory_copy_trace.csv.gz"
      cat "$O/trace_bench.json" ;;
    pmc)
      # each (config, grid) with the grid fixed (MXEC_RS_BPC also turns the
      # grid tuner off), counters only on rs_apply_fast, one run per counter
      for cb in 2:1024 2:512 2:256 ns:512 ns:256 ns:128; do
        cfg=${cb%%:*}; bpc=${cb##*:}
        for c in FETCH_SIZE WRITE_SIZE; do
          ( cd /tmp && MXEC_LIB="$R/maxio_amd/lib/libmaxio_ec_lab.so" MXEC_RS_BPC=$bpc timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex rs_apply_fast \
              -d "/tmp/pmc/${cfg}_${bpc}_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 2 \
              --warmup 1 --cpu-seconds 0 --no-extra --no-e2e > "$O/pmc_${cfg}_${bpc}_$c.log" 2>&1 ) \
              || { tail -5 "$O/pmc_${cfg}_${bpc}_$c.log"; exit 1; }
          find "/tmp/pmc/${cfg}_${bpc}_$c" -name "*counter_collection.csv" -exec cp {} "$O/pmc_${cfg}_${bpc}_$c.csv" \;
        done
      done
      # configs[1]: 1024 x 4+2 x 10 MiB = 655 360 tiles of 16 KiB;
      # north star: 4096 x 8+4 x 1 MiB = 262 144 tiles.
      for cb in 2:1024 2:512 2:256; do
        bpc=${cb##*:}
        python tools/pmc_summary.py "$O/pmc_2_${bpc}_FETCH_SIZE.csv" "$O/pmc_2_${bpc}_WRITE_SIZE.csv" \
          "rs_apply_fast<2, 4, true, false" 64424509440 --blocks-per-cu $bpc --tiles 655360 \
          --what "config 2, rs_apply_fast<2,4,nt> at $bpc WG/CU" --out "$O/pmc_k4m2_bpc${bpc}_traffic.json" || exit 1
      done
      for cb in ns:512 ns:256 ns:128; do
        bpc=${cb##*:}
        python tools/pmc_summary.py "$O/pmc_ns_${bpc}_FETCH_SIZE.csv" "$O/pmc_ns_${bpc}_WRITE_SIZE.csv" \
          "rs_apply_fast<4, 4, true, false" 51539607552 --blocks-per-cu $bpc --tiles 262144 \
          --what "north star, rs_apply_fast<4,4,nt> at $bpc WG/CU" --out "$O/pmc_k8m4_bpc${bpc}_traffic.json" || exit 1
      done ;;
    clock)
      for cfg in 3 2 ns; do
        ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT \
            --kernel-include-regex 'sha256|rs_apply' -d "/tmp/clk/$cfg" -o run --output-format csv \
            -- python3 "$R/bench.py" --config $cfg --steps 3 --warmup 1 --cpu-seconds 0 --no-extra --no-e2e \
            > "$O/clock_$cfg.log" 2>&1 ) || { tail -5 "$O/clock_$cfg.log"; exit 1; }
        find "/tmp/clk/$cfg" -name "*counter_collection.csv" -exec cp {} "$O/clock_$cfg.csv" \;
        python tools/clock_summary.py "$O/clock_$cfg.csv" --what "bench.py --config $cfg, GRBM pass" \
          --out "$O/clock_$cfg.json" || exit 1
      done ;;
    rust)
      { command -v rustc; command -v cargo; rustc --version; cargo --version; } > "$O/rust_probe.txt" 2>&1 || true
      cat "$O/rust_probe.txt" ;;
    pyt:*)
      IFS=+ read -ra F <<< "${st#pyt:}"
      files=(); for f in "${F[@]}"; do files+=("tests/$f.py"); done
      timeout -k 10 900 python -u -m pytest "${files[@]}" -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/pytest_${F[0]}.log" 2>&1 || { tail -40 "$O/pytest_${F[0]}.log"; exit 1; }
      tail -2 "$O/pytest_${F[0]}.log" ;;
    tool:*)
      t="${st#tool:}"; v="TOOL_ARGS_$t"; targs="${!v:-$TOOL_ARGS}"
      timeout -k 10 "${TOOL_TIMEOUT:-600}" python -u "tools/$t.py" $targs > "$O/$t.jsonl" 2> "$O/$t.err" \
        || { tail -20 "$O/$t.err"; exit 1; }
      cat "$O/$t.jsonl" ;;
    pmc5)
      # config 5's step (grouped / multi-r launches) under FETCH_SIZE and
      # WRITE_SIZE passes, one run each: 1 warmup + 3 timed steps
      for c in FETCH_SIZE WRITE_SIZE; do
        ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex rs_apply -d "/tmp/pmc5/$c" -o run \
            --output-format csv -- python3 "$R/bench.py" --config 5 --steps 3 --warmup 1 --cpu-seconds 0 --no-extra \
            --no-e2e > "$O/pmc5_$c.log" 2>&1 ) || { tail -5 "$O/pmc5_$c.log"; exit 1; }
        find "/tmp/pmc5/$c" -name "*counter_collection.csv" -exec cp {} "$O/pmc5_$c.csv" \;
      done
      python tools/pmc_step_summary.py "$O/pmc5_FETCH_SIZE.csv" "$O/pmc5_WRITE_SIZE.csv" "$O/pmc5_FETCH_SIZE.log" \
        --blocks-per-cu 512 --out "$O/r6_pmc_cfg5_grouped_traffic.json" || exit 1 ;;
    exitprobe)
      # one pageable host batch under the profiler options
      # whose teardown faulted in round 5 (tools/exit_probe.py).  Run it last:
      # a non-zero exit (139) ends the call.
      ( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/exitprobe -o run \
          --output-format csv -- python3 "$R/tools/exit_probe.py" host_pageable > "$O/exit_pageable.out" \
          2> "$O/exit_pageable.err" ); rc=$?
      echo "{\"what\": \"host_pageable under rocprofv3 --kernel-trace --memory-copy-trace\", \"rc\": $rc}" \
        | tee -a "$O/exit_probe.jsonl"
      [ "$rc" = 0 ] || exit 1 ;;
    cfg:*)
      c="${st#cfg:}"
      timeout -k 10 900 python bench.py --config "$c" --no-extra $BENCH_ARGS > "$O/cfg_$c.json" 2> "$O/cfg_$c.err" || { tail -20 "$O/cfg_$c.err"; exit 1; }
      cat "$O/cfg_$c.json" ;;
    *) echo "unknown step $st"; exit 1 ;;
  esac
done
echo "== done $(date +%T)"
