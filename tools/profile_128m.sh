#!/bin/bash
# Kernel trace of the 128M x 128M config (launch / host overhead check).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p128m -o run --output-format csv -- python $R/bench.py --inner 1.28e8 --outer 1.28e8 --steps 20 --warmup 3 --general off > $R/gpurun_out/p128m.log 2>&1 && echo done
