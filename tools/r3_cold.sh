#!/bin/bash
# Cold-join investigation: VRAM reuse probe, then the default bench (headline
# + general path in one process) with the arena trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/r3b
timeout -k 10 120 python -u tools/vram_reuse_probe.py > gpurun_out/r3b/vram_reuse.jsonl 2>&1 || { tail -20 gpurun_out/r3b/vram_reuse.jsonl; exit 1; }
HPCJOIN_TRACE_ALLOC=1 HPCJOIN_TRACE_FIRST=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3b/bench_trace.log 2>&1 || { tail -20 gpurun_out/r3b/bench_trace.log; exit 1; }
echo done
