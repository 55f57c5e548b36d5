#!/bin/bash
# Kernel trace of one rank's share of the N = 8 headline (125M x 125M) and a
# plain bench of the same size: the fixed per-join cost that strong scaling
# exposes.  Also the 1B x 1B kernel stats of the current tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-rank8}
timeout -k 10 300 python $R/bench.py --inner 1.25e8 --outer 1.25e8 --steps 20 --warmup 3 --general off > $R/gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 $R/gpurun_out/${TAG}_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p125m -o run --output-format csv -- python $R/bench.py --inner 1.25e8 --outer 1.25e8 --steps 20 --warmup 3 --general off > $R/gpurun_out/${TAG}_p125m.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_p125m.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p1b -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/${TAG}_p1b.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_p1b.log; exit 1; }
echo done
