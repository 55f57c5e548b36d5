#!/bin/bash
# Replicated-bitmap plan with the all-reduce in partition ranges: full GPU
# suite (in-process and RCCL multi-process ranks), 8 in-process ranks at 1B
# with 1 and 4 ranges, and the 8-process RCCL bench on the shared GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-rc}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for k in 1 4; do
  HPCJOIN_REDUCE_CHUNKS=$k timeout -k 10 200 python tools/rehearse_inprocess.py --ranks 8 --size 1e9 > gpurun_out/${TAG}_inproc8_k$k.log 2>&1 || { tail -20 gpurun_out/${TAG}_inproc8_k$k.log; exit 1; }
  echo "k=$k $(grep -o '"ok": [a-z]*' gpurun_out/${TAG}_inproc8_k$k.log | head -1) $(grep -o '"join_ms": [0-9.]*' gpurun_out/${TAG}_inproc8_k$k.log | head -1)"
done
HPCJOIN_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --inner 1e8 --outer 1e8 --steps 3 --warmup 1 --general off > gpurun_out/${TAG}_8proc.log 2>&1 || { tail -20 gpurun_out/${TAG}_8proc.log; exit 1; }
tail -1 gpurun_out/${TAG}_8proc.log | cut -c1-600
echo done
