#!/bin/bash
# Round 5: verified GET in pipelined verification groups and the probe-driven
# copy engine.  Tests first, then the e2e GET sizes (auto), the one-group
# form (lab build, MXEC_GET_VGROUPS=1) and wave copies at 512 objects, then
# the driver's bench command (its post-extras GET leg), then whether
# rocprofv3's memory-copy trace crashes at exit on a torch-only program.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5b}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_get_groups_gpu.py \
  tests/test_pipeline_2d_gpu.py tests/test_coef_arena_gpu.py tests/test_pipeline_gpu.py tests/test_contract_gpu.py \
  > $out/pytest_sel.log 2>&1 || { tail -30 $out/pytest_sel.log; exit 1; }
tail -1 $out/pytest_sel.log
for n in 128 256 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned --get \
    > $out/e2e_$n.json 2> $out/e2e_$n.err || { tail -5 $out/e2e_$n.err; exit 1; }
done
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_GET_VGROUPS=1 timeout -k 10 300 python -u tools/e2e_bench.py \
  --objects 512 --reps 3 --alloc mxec --modes pinned --get > $out/e2e_512_one_group.json 2> $out/e2e_512_one_group.err \
  || { tail -5 $out/e2e_512_one_group.err; exit 1; }
MXEC_PIPE_COPY=waves timeout -k 10 300 python -u tools/e2e_bench.py --objects 512 --reps 3 --alloc mxec --modes pinned \
  --get > $out/e2e_512_waves.json 2> $out/e2e_512_waves.err || { tail -5 $out/e2e_512_waves.err; exit 1; }
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err \
  || { tail -20 $out/bench.err; exit 1; }
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so timeout -k 10 600 python -u tools/placement_lab.py --objects 1024 \
  --allocs 5 --free-each --spacer-mib 0,6144,12288,20480,30720 --grids 1024 --lds 2:512,2:1024,4:256,4:512 --reps 5 \
  > $out/placement_lds.jsonl 2> $out/placement_lds.err || { tail -5 $out/placement_lds.err; exit 1; }
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tc -o run --output-format csv \
    -- python3 -c "import torch; x = torch.ones(1 << 20, device='cuda'); print(float(x.cpu().sum()))" \
    > "$OLDPWD/$out/trace_torch_only.out" 2> "$OLDPWD/$out/trace_torch_only.err" ); echo "torch-only trace exit $?" | tee $out/trace_torch_only.rc
