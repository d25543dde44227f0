#!/bin/bash
# Pinned host buffers bound to the GPU's NUMA node (mxec_host_alloc) or not:
# the pipeline GPU tests, then the bench's e2e leg in fresh processes
# alternating MXEC_HOST_NUMA=1/0 after one discarded warm process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${1:?out subdir}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest_pipeline.log" 2>&1 || { tail -30 "$O/pytest_pipeline.log"; exit 1; }
tail -1 "$O/pytest_pipeline.log"
timeout -k 10 200 python tools/e2e_reps.py --runs 1 > "$O/warm.jsonl" 2> "$O/warm.err" || { tail -5 "$O/warm.err"; exit 1; }
for r in 1 2 3; do
  for v in 1 0; do
    MXEC_HOST_NUMA=$v timeout -k 10 200 python tools/e2e_reps.py --runs 1 >> "$O/numa_ab.jsonl" 2>> "$O/numa_ab.err" \
      || { tail -5 "$O/numa_ab.err"; exit 1; }
  done
done
cat "$O/numa_ab.jsonl"
