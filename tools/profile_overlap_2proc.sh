#!/bin/bash
# Kernel trace of 2 RCCL processes sharing the GPU (1B x 1B, replicated plan):
# shows the ranged all-reduce kernels on the exchange stream overlapping the
# outer side's scatter on the compute stream (socket transport: the
# all-reduce itself is slow here).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-ov2}
HPCJOIN_SHARE_GPU=1 timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG} -o run --output-format csv -- python $R/bench.py --gpus 2 --steps 2 --warmup 1 --general off > $R/gpurun_out/${TAG}.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}.log; exit 1; }
ls -R $R/gpurun_out/${TAG} | head -20
echo done
