#!/bin/bash
# General path after moving its sampled slice layout to the device: full GPU
# tests, general-path bench x2 and a kernel trace (per-join idle time).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3d}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
bash tools/ab_bench.sh $TAG general "" "" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $R/bench.py --general only --steps 3 --warmup 1 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
echo done
