#!/bin/bash
# A/B of the fused row-output kernel's occupancy: default plan (1024-tuple
# chunks, 3 blocks per CU) vs 512-tuple chunks (5 blocks per CU).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
timeout -k 10 300 python $R/tools/bench_tpch.py --steps 4 --warmup 1 > $R/gpurun_out/rows_A.log 2>&1 || exit 1
HPCJOIN_BUILD_TARGET=512 HPCJOIN_R_CHUNK=512 timeout -k 10 300 python $R/tools/bench_tpch.py --steps 4 --warmup 1 > $R/gpurun_out/rows_B.log 2>&1 || exit 1
HPCJOIN_BUILD_TARGET=512 HPCJOIN_R_CHUNK=1024 timeout -k 10 300 python $R/tools/bench_tpch.py --steps 4 --warmup 1 > $R/gpurun_out/rows_C.log 2>&1 || exit 1
echo done
