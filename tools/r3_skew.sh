#!/bin/bash
# Skew configurations with the exact per-key oracle: a small sanity pass, the
# 1B x 4B single-GPU configs, then a 4-rank shared-GPU rehearsal of the
# assignment variants.  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3s}; mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u tools/bench_skew.py --inner 1e7 --outer 4e7 > gpurun_out/$TAG/skew_small.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/skew_small.jsonl; exit 1; }
cut -c1-300 gpurun_out/$TAG/skew_small.jsonl
timeout -k 10 500 python -u tools/bench_skew.py --inner 1e9 --outer 4e9 > gpurun_out/$TAG/skew_1b_4b.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/skew_1b_4b.jsonl; exit 1; }
cut -c1-400 gpurun_out/$TAG/skew_1b_4b.jsonl
HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python -u tools/bench_skew.py --gpus 4 --inner 1e8 --outer 4e8 --configs zipf_both --assign lpt,round_robin --split on,off > gpurun_out/$TAG/skew_4rank.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/skew_4rank.jsonl; exit 1; }
cut -c1-300 gpurun_out/$TAG/skew_4rank.jsonl
echo done
