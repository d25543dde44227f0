#!/bin/bash
# Wave copies with CU-masked streams: the copy-mode test, then the default
# bench with MXEC_PIPE_COPY=waves at 32 (default) and 16 copy CUs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4i}
mkdir -p "$O"
export TMPDIR=/tmp
LAB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for v in waves:16 waves:32 waves2:16; do
  mode=${v%%:*}; g=${v##*:}
  MXEC_PIPE_COPY=$mode MXEC_PIPE_COPY_GRID=$g MXEC_LIB=$LAB MXEC_PIPE_TRACE=1 timeout -k 10 400 python bench.py --cpu-seconds 1 \
    > "$O/bench_${mode}_grid$g.json" 2> "$O/bench_${mode}_grid$g.err" || { tail -20 "$O/bench_${mode}_grid$g.err"; exit 1; }
done
echo done
