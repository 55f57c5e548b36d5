#!/bin/bash
# First-join cost with eager code-object loading (HIP_ENABLE_DEFERRED_LOADING=0) vs default.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3f}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for v in 1 0 1 0; do
  t0=$(date +%s.%N)
  HIP_ENABLE_DEFERRED_LOADING=$v HPCJOIN_TRACE_FIRST=1 timeout -k 10 200 python -u bench.py --general off --steps 3 --warmup 1 > $OUT/defer$v.log 2>&1 || { tail -20 $OUT/defer$v.log; exit 1; }
  t1=$(date +%s.%N)
  echo "deferred=$v wall $(echo "$t1 - $t0" | bc) s: $(grep first_join $OUT/defer$v.log | cut -c1-60) $(grep -o '"first_ms": [0-9.]*' $OUT/defer$v.log)"
done
