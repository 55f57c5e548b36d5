#!/bin/bash
# Multi-process rehearsal of the N-GPU bench on a 1-GPU box: N ranks share the
# device (HPCJOIN_SHARE_GPU=1, RCCL socket transport).  Exchange times are NOT
# xGMI times; this checks the RCCL path end to end at full scale.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
N=${1:-2}; SIZE=${2:-1e8}; TAG=${3:-rehearse}
export HPCJOIN_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port $((29500 + N)) bench.py --gpus $N --inner $SIZE --outer $SIZE --steps 3 --warmup 1 \
  > gpurun_out/${TAG}_n${N}.log 2>&1; rc=$?
grep '^{' gpurun_out/${TAG}_n${N}.log || tail -30 gpurun_out/${TAG}_n${N}.log
exit $rc
