#!/bin/bash
# Shared timeline points on the two-level path: full GPU suite, then the
# general path at 125M / 1B with the timeline on and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-pt2}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for size in 1.25e8 1e9; do
  for tl in 1 0; do
    L=gpurun_out/${TAG}_${size}_${tl}.log
    HPCJOIN_TIMELINE=$tl timeout -k 10 200 python bench.py --inner $size --outer $size --general only --steps 10 --warmup 2 > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'timeline', sys.argv[3], d['ms_per_step'], d['correct'])" $L $size $tl
  done
done
