#!/bin/bash
# TPC-H SF100 late materialization variants (HPCJOIN_MAT_VARIANT).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  HPCJOIN_MAT_VARIANT=$v timeout -k 10 300 python tools/bench_tpch.py --steps 3 --warmup 1 > gpurun_out/mat_v$v.log 2>&1 || { tail -5 gpurun_out/mat_v$v.log; exit 1; }
  echo "variant $v $(tail -1 gpurun_out/mat_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["median_total_ms"], d["median_join_ms"], d["median_materialize_ms"], d["correct"])')"
done
