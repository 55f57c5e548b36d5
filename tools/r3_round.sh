#!/bin/bash
# Default bench (headline + general path), then a 2-rank shared-GPU RCCL
# rehearsal of the N > 1 record (topology, link calibration, shuffle_path).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3r}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/$TAG/bench.log 2>&1 || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["general_path"]; print("head", d["ms_per_step"], d["first_join_ms"], d["setup_ms"], d["correct"], "general", g.get("ms_per_step"), g.get("first_join_ms"), g.get("setup_ms"), g.get("correct"))'
HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --inner 2e8 --outer 2e8 --steps 3 --warmup 1 > gpurun_out/$TAG/rehearsal2.log 2>&1 || { tail -20 gpurun_out/$TAG/rehearsal2.log; exit 1; }
tail -1 gpurun_out/$TAG/rehearsal2.log | cut -c1-400
echo done
