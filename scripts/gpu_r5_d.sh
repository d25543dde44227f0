#!/bin/bash
# Round 5: the full GPU suite (two producer waves in the lag pair SHA-256
# form, non-blocking SDMA watch); the SHA-256 producer question (config 3:
# the schedule-free diagnostic build -- how fast the lag pair consumers run
# when the producer is never late --, the new two-lane producers, the old
# one-wave producer); verification groups re-measured; the driver's bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5d}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
  > $out/pytest_sel.log 2>&1 || { tail -30 $out/pytest_sel.log; exit 1; }
tail -1 $out/pytest_sel.log
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab_nosched.so timeout -k 10 300 python bench.py --config 3 --no-extra --no-e2e \
  --cpu-seconds 0 --steps 10 --warmup 3 > $out/cfg3_nosched.json 2> $out/cfg3_nosched.err || { tail -5 $out/cfg3_nosched.err; exit 1; }
timeout -k 10 300 python bench.py --config 3 --no-extra --no-e2e --cpu-seconds 0 --steps 10 --warmup 3 \
  > $out/cfg3.json 2> $out/cfg3.err || { tail -5 $out/cfg3.err; exit 1; }
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_SHA_PRODUCERS=1 timeout -k 10 300 python bench.py --config 3 \
  --no-extra --no-e2e --cpu-seconds 0 --steps 10 --warmup 3 > $out/cfg3_one_producer.json 2> $out/cfg3_one_producer.err \
  || { tail -5 $out/cfg3_one_producer.err; exit 1; }
for n in 128 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned --get \
    > $out/e2e_$n.json 2> $out/e2e_$n.err || { tail -5 $out/e2e_$n.err; exit 1; }
done
for g in 1 2 4; do
  MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_GET_VGROUPS=$g timeout -k 10 300 python -u tools/e2e_bench.py \
    --objects 512 --reps 3 --alloc mxec --modes pinned --get > $out/e2e_512_g$g.json 2> $out/e2e_512_g$g.err \
    || { tail -5 $out/e2e_512_g$g.err; exit 1; }
done
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err \
  || { tail -20 $out/bench.err; exit 1; }
echo done
