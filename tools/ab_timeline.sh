#!/bin/bash
# What the device sub-phase timing events cost inside a join: 1B and 125M
# with HPCJOIN_TIMELINE=0 (no Timeline events) vs the default, alternated.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-tl}
for rep in 1 2; do
for size in 1.25e8 1e9; do
  for tl in 1 0; do
    L=gpurun_out/${TAG}_${size}_${tl}_${rep}.log
    HPCJOIN_TIMELINE=$tl timeout -k 10 200 python bench.py --inner $size --outer $size --steps 20 --warmup 3 --general off > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'timeline', sys.argv[3], d['ms_per_step'], d['correct'])" $L $size $tl
  done
done
done
cd /tmp && export TMPDIR=/tmp
HPCJOIN_TIMELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p125m -o run --output-format csv -- python $R/bench.py --inner 1.25e8 --outer 1.25e8 --steps 20 --warmup 3 --general off > $R/gpurun_out/${TAG}_p125m.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_p125m.log; exit 1; }
echo done
