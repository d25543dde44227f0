#!/bin/bash
# Piece-major host PUT pipeline: GPU tests of the host pipeline, then the
# within-process A/B (tools/e2e_piece_ab.py).  Each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${1:?out subdir}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_gpu_parity.py -k "batch_host or sha256" -x -v \
  --timeout 120 --timeout-method thread > "$O/pytest_pieces.log" 2>&1 || { tail -40 "$O/pytest_pieces.log"; exit 1; }
tail -1 "$O/pytest_pieces.log"
timeout -k 10 300 python tools/e2e_piece_ab.py --values 0,1,2 --rounds 3 --get > "$O/piece_ab.jsonl" 2> "$O/piece_ab.err" \
  || { tail -20 "$O/piece_ab.err"; exit 1; }
cat "$O/piece_ab.jsonl"
timeout -k 10 300 python tools/e2e_piece_ab.py --values 0,1 --rounds 2 --no-digests > "$O/piece_ab_nodig.jsonl" 2> "$O/piece_ab_nodig.err" \
  || { tail -20 "$O/piece_ab_nodig.err"; exit 1; }
cat "$O/piece_ab_nodig.jsonl"
