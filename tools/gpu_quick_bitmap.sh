#!/bin/bash
# Bitmap-plan check: bitmap + distributed GPU tests, 1B bench, 8-process RCCL
# rehearsal on the shared GPU (100M).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-qb}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "bitmap or Bitmap or distributed or rccl" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --general off > gpurun_out/${TAG}_1b.log 2>&1 || { tail -20 gpurun_out/${TAG}_1b.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('1b', d['ms_per_step'], d['value'], d['correct'])" gpurun_out/${TAG}_1b.log
HPCJOIN_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 8 --inner 1e8 --outer 1e8 --steps 3 --warmup 1 --general off > gpurun_out/${TAG}_8proc.log 2>&1 || { tail -20 gpurun_out/${TAG}_8proc.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('8proc', d['ms_per_step'], d['correct'], d['config']['plan'])" gpurun_out/${TAG}_8proc.log
echo done
