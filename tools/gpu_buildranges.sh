#!/bin/bash
# Build ranges feeding the ranged all-reduce: bitmap + distributed GPU tests,
# 1B over 2 RCCL processes sharing the GPU, 8 in-process ranks at 1B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-br}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "bitmap or Bitmap or distributed or rccl or measurement" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --general off > gpurun_out/${TAG}_2proc.log 2>&1 || { tail -20 gpurun_out/${TAG}_2proc.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('2proc', d['ms_per_step'], d['correct'], d['matches'])" gpurun_out/${TAG}_2proc.log
timeout -k 10 200 python tools/rehearse_inprocess.py --ranks 8 --size 1e9 > gpurun_out/${TAG}_inproc8.log 2>&1 || { tail -20 gpurun_out/${TAG}_inproc8.log; exit 1; }
grep -o '"ok": [a-z]*' gpurun_out/${TAG}_inproc8.log | head -1
echo done
