#!/bin/bash
# Round 5 numbers of record at HEAD: the GPU suite and smoke, the driver's
# bench command, the same under rocprofv3 (kernel stats + the headline's
# timed launches), then the verified GET's verification groups traced (lab
# build, MXEC_PIPE_TRACE=1: where G = 2 loses), then the profiler-exit probe
# series (last: it stops at the first run that does not exit 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5e}
mkdir -p $out
export TMPDIR=/tmp
R=$PWD
bash scripts/gpu.sh ${1:-r5e} tests,smoke,bench,prof || exit 1
for g in 1 2 4; do
  MXEC_LIB=$R/maxio_amd/lib/libmaxio_ec_lab.so MXEC_GET_VGROUPS=$g MXEC_PIPE_TRACE=1 timeout -k 10 300 \
    python -u tools/e2e_bench.py --objects 512 --reps 2 --alloc mxec --modes pinned --get \
    > $out/trace_g$g.json 2> $out/trace_g$g.err || { tail -5 $out/trace_g$g.err; exit 1; }
done
bash scripts/gpu_r5_exit.sh ${1:-r5e}
echo "exit probe series: $?"
