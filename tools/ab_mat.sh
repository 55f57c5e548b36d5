#!/bin/bash
# A/B of materializeLocalKernel variants (HPCJOIN_MAT_VARIANT 0..3) on the SF100 TPC-H bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
for v in 0 1 2 3; do
  HPCJOIN_MAT_VARIANT=$v timeout -k 10 200 python $R/tools/bench_tpch.py --steps 3 --warmup 1 > $R/gpurun_out/abmat_$v.log 2>&1 || exit 1
  echo "variant $v: $(grep -o '"median_materialize_ms": [0-9.]*' $R/gpurun_out/abmat_$v.log)"
done
