#!/bin/bash
# Round-3 first look: MALL residency probe, cold general join with the arena
# trace, kernel stats of the general path.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r3a
timeout -k 10 180 python -u tools/mall_probe.py > gpurun_out/r3a/mall_probe.jsonl 2>&1 || { tail -20 gpurun_out/r3a/mall_probe.jsonl; exit 1; }
HPCJOIN_TRACE_ALLOC=1 timeout -k 10 300 python -u bench.py --general only --steps 5 --warmup 2 > gpurun_out/r3a/general_trace.log 2>&1 || { tail -20 gpurun_out/r3a/general_trace.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3a/stats -o run --output-format csv -- python $R/bench.py --general only --steps 3 --warmup 1 > $R/gpurun_out/r3a/stats.log 2>&1 || { tail -20 $R/gpurun_out/r3a/stats.log; exit 1; }
echo done
