#!/bin/bash
# 2-process shared-GPU bench.py: sampled vs exact N > 1 network pass
# (HPCJOIN_NETWORK_HISTOGRAM=EXACT).  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3q}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for mode in AUTO EXACT AUTO EXACT; do
  HPCJOIN_NETWORK_HISTOGRAM=$mode HPCJOIN_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --inner 2e8 --outer 2e8 --steps 3 --warmup 1 > $OUT/ab_$mode.log 2>&1 || { tail -20 $OUT/ab_$mode.log; exit 1; }
  grep '^{' $OUT/ab_$mode.log | python3 -c '
import json,sys; d=json.loads(sys.stdin.read())
print(sys.argv[1], "head", d["ms_per_step"], *[(k, d[k]["ms_per_step"], d[k]["correct"], d[k]["sampled_network"], d[k]["phases_ms"]["dev_network_ms"]) for k in ("shuffle_path","general_path")])' $mode
done
