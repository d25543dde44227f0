#!/bin/bash
# Cut tiles inside the fast RS kernel: the new parity sweeps, the whole GPU
# suite, then small-chunk lab and config 5, new vs previous library (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2ai; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cut_tiles_gpu.py -x -q --timeout 120 --timeout-method thread > $O/cut.log 2>&1 || { tail -30 $O/cut.log; exit 1; }
tail -2 $O/cut.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for lib in new old; do
  if [ $lib = old ]; then export MXEC_LIB=$PWD/build_ab/libmaxio_ec_edge.so; else unset MXEC_LIB; fi
  timeout -k 10 300 python tools/small_chunk_lab.py --km 8,4 > $O/lab_$lib.jsonl 2> $O/lab_$lib.err || { tail -20 $O/lab_$lib.err; exit 1; }
  echo "== $lib"; cut -c1-200 $O/lab_$lib.jsonl
done
for r in 1 2; do for lib in new old; do
  if [ $lib = old ]; then export MXEC_LIB=$PWD/build_ab/libmaxio_ec_edge.so; else unset MXEC_LIB; fi
  timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-extra --cpu-seconds 0 > $O/b5_${lib}_$r.json 2> $O/b5_${lib}_$r.err || { tail $O/b5_${lib}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b5_${lib}_$r.json')); print('$lib', $r, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['spot_check_vs_oracle'])"
done; done
