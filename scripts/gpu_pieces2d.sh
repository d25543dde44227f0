#!/bin/bash
# 2D piece copies and the piece ramp: host-pipeline GPU tests, then
# within-process A/Bs (tools/e2e_piece_ab.py) of MXEC_PIPE_COPY2D and, with
# 2D copies on, MXEC_PIPE_RAMP_KB.  Each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${1:?out subdir}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_pipeline.log" 2>&1 || { tail -40 "$O/pytest_pipeline.log"; exit 1; }
tail -1 "$O/pytest_pipeline.log"
timeout -k 10 300 python tools/e2e_piece_ab.py --env MXEC_PIPE_COPY2D --values 0,1 --rounds 3 --get \
  > "$O/copy2d_ab.jsonl" 2> "$O/copy2d_ab.err" || { tail -20 "$O/copy2d_ab.err"; exit 1; }
cat "$O/copy2d_ab.jsonl"
MXEC_PIPE_COPY2D=1 timeout -k 10 300 python tools/e2e_piece_ab.py --env MXEC_PIPE_RAMP_KB --values 0,64,256 --rounds 3 --get \
  > "$O/ramp_ab.jsonl" 2> "$O/ramp_ab.err" || { tail -20 "$O/ramp_ab.err"; exit 1; }
cat "$O/ramp_ab.jsonl"
