#!/bin/bash
# Every single-GPU config on the current tree (tools/bench_configs.sh) plus the
# skew configs with duplicate inner keys and 3B x 3B / 4B x 4B capacity runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3cfg}; mkdir -p gpurun_out/$TAG
bash tools/bench_configs.sh $TAG/cfg || exit 1
timeout -k 10 600 python -u tools/bench_skew.py --configs zipf_both,uniform_two > gpurun_out/$TAG/skew.jsonl 2> gpurun_out/$TAG/skew.err || { tail -5 gpurun_out/$TAG/skew.err; exit 1; }
tail -2 gpurun_out/$TAG/skew.jsonl | cut -c1-300
timeout -k 10 400 python -u bench.py --inner 3e9 --outer 3e9 --steps 3 --warmup 1 --general off > gpurun_out/$TAG/3b.log 2>&1 || { tail -5 gpurun_out/$TAG/3b.log; exit 1; }
echo "3b $(tail -1 gpurun_out/$TAG/3b.log | cut -c1-300)"
