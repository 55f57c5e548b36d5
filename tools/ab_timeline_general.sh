#!/bin/bash
# Timing-event cost on the general (two-level, key-only) path: timeline on/off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-tlg}
for rep in 1 2; do
for size in 1.25e8 1e9; do
  for tl in 1 0; do
    L=gpurun_out/${TAG}_${size}_${tl}_${rep}.log
    HPCJOIN_TIMELINE=$tl timeout -k 10 200 python bench.py --inner $size --outer $size --general only --steps 10 --warmup 2 > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'timeline', sys.argv[3], d['ms_per_step'], d['correct'])" $L $size $tl
  done
done
done
