set -o pipefail
R=$(pwd); O=$R/gpurun_out/r3pmcsha; mkdir -p $O
( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex sha256_quad \
    -d /tmp/pmcsha -o run --output-format csv -- python3 "$R/bench.py" --config 3 --steps 2 --warmup 1 --cpu-seconds 0 --no-extra --no-e2e \
    > $O/pmc.log 2>&1 ) || { tail -5 $O/pmc.log; exit 1; }
find /tmp/pmcsha -name "*counter_collection.csv" -exec cp {} $O/counters.csv \;
find /tmp/pmcsha -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \; || true
wc -l $O/counters.csv
