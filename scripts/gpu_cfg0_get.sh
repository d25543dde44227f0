set -o pipefail
O=gpurun_out/r3cfg0; mkdir -p $O
for W in 1 16 128; do
  timeout -k 10 300 python tools/e2e_get_bench.py --k 1 --parity 2 --chunk-size 10485760 --erasures 1 --threads $W --objects $((W>8?W:8)) --cpu-objects 8 > $O/get_w$W.json 2> $O/get_w$W.err || { tail -5 $O/get_w$W.err; exit 1; }
  cat $O/get_w$W.json
done
timeout -k 10 300 python tools/get_latency.py > $O/latency.json 2> $O/latency.err || { tail -5 $O/latency.err; exit 1; }
cat $O/latency.json
