set -o pipefail
mkdir -p gpurun_out/r3q
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sha256" -x -v --timeout 120 --timeout-method thread > gpurun_out/r3q/pytest_sha.log 2>&1 || { tail -40 gpurun_out/r3q/pytest_sha.log; exit 1; }
tail -3 gpurun_out/r3q/pytest_sha.log
timeout -k 10 300 python tools/sha_split_ab.py --env MXEC_SHA_FORM --values quad,split --messages 10240 > gpurun_out/r3q/ab_cfg3.jsonl 2>&1 || { tail -20 gpurun_out/r3q/ab_cfg3.jsonl; exit 1; }
cat gpurun_out/r3q/ab_cfg3.jsonl
timeout -k 10 300 python tools/sha_split_ab.py --env MXEC_SHA_FORM --values quad,split --messages 3 --size 10485760 --rounds 2 --reps 2 > gpurun_out/r3q/ab_10m.jsonl 2>&1 || { tail -20 gpurun_out/r3q/ab_10m.jsonl; exit 1; }
cat gpurun_out/r3q/ab_10m.jsonl
bash scripts/gpu.sh r3q tests,smoke
