#!/bin/bash
# Is one config-2 launch short of the chip? Same box, three alternating
# rounds: 1 rank, 1 rank with the batch as 2 / 4 launches on their own
# streams, 2 ranks sharing the GPU (gloo).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2u; mkdir -p $O
for r in 1 2 3; do
 for ns in 1 2 4; do
  BENCH_ENCODE_STREAMS=$ns timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extra > $O/s${ns}_$r.json 2> $O/s${ns}_$r.err || { tail -20 $O/s${ns}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s${ns}_$r.json')); r=d['roofline']; print('round $r streams $ns', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream_GBps'), d['spot_check_vs_oracle'])"
 done
 BENCH_GPU_OF_RANK=0 BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-seconds 0 > $O/ranks2_$r.json 2> $O/ranks2_$r.err || { tail -30 $O/ranks2_$r.err; exit 1; }
 python -c "
import json
line = [l for l in open('$O/ranks2_$r.json') if l.lstrip().startswith('{')][-1]
d = json.loads(line); print('round $r 2 ranks', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
