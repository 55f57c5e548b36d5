#!/bin/bash
# The driver's N = 8 headline invocation shape on one GPU: 8 RCCL processes
# (socket transport, shared GPU), 1B x 1B, replicated plan + general path.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-r8}
HPCJOIN_SHARE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/${TAG}.log 2>&1 || { tail -30 gpurun_out/${TAG}.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['general_path']; print('8proc', d['ms_per_step'], d['correct'], d['matches'], d['config']['parallelism'], 'general', g.get('ms_per_step'), g.get('correct'), g.get('matches'))" gpurun_out/${TAG}.log
