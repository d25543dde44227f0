#!/bin/bash
# SHA-256 stream form: correctness of the production build against the split
# form (tools/sha_stream_lab check: digests + work words), then the big-batch
# timings beside the split / one-wave forms, then the stream GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2e; mkdir -p $O
echo "== lab check"; timeout -k 5 60 tools/sha_stream_lab check > $O/lab_check.jsonl 2>&1; rc=$?
grep -v "items (" $O/lab_check.jsonl | cut -c1-220; echo "rc=$rc"; [ $rc -eq 0 ] || exit 1
echo "== lab big"; timeout -k 5 240 tools/sha_stream_lab big > $O/lab_big.jsonl 2>&1 || { cat $O/lab_big.jsonl; exit 1; }
cat $O/lab_big.jsonl
echo "== stream tests"
timeout -k 10 400 python -u -m pytest tests/test_sha_stream_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -30 $O/pytest_stream.log; exit 1; }
tail -3 $O/pytest_stream.log
