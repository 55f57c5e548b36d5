#!/bin/bash
# A/B of the key-only count kernel variants (HPCJOIN_KCOUNT) on the general path.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
for v in ${VARIANTS:-0 1 2 3 4 5}; do
  HPCJOIN_KCOUNT=$v timeout -k 10 200 python $R/bench.py --general only --steps 8 --warmup 2 > $R/gpurun_out/kc_$v.log 2>&1 || exit 1
done
echo done
