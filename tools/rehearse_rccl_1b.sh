#!/bin/bash
# 1B x 1B over 2 and 4 RCCL processes sharing the one GPU (socket transport):
# the replicated plan with its all-reduce in 4 partition ranges through real
# RCCL; correctness, not link speed.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-rr}
for n in 2 4; do
  HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus $n --steps 3 --warmup 1 --general off > gpurun_out/${TAG}_${n}.log 2>&1 || { tail -20 gpurun_out/${TAG}_${n}.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ranks', d['ms_per_step'], d['correct'], d['matches'], d['config']['parallelism'], d['links']['measured_wire_bytes_rank0'])" gpurun_out/${TAG}_${n}.log $n
done
echo done
