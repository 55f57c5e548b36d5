#!/bin/bash
# rocprofv3 kernel stats of the SF100 TPC-H-like bench (join + late materialization).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-tpch_prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG} -o run --output-format csv -- python $R/tools/bench_tpch.py --steps 3 --warmup 1 > $R/gpurun_out/${TAG}.log 2>&1 && echo done
