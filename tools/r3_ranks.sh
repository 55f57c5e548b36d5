#!/bin/bash
# Multi-process rehearsals on the one GPU (HPCJOIN_SHARE_GPU=1, RCCL socket
# transport): RCCL worker tests (incl. TPC-H), TPC-H SF10 at 2 and 4 ranks,
# bench.py at 2 ranks, skew assignment variants at 8 ranks.  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3m}; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py -k rccl_multiprocess > gpurun_out/$TAG/rccl_tests.log 2>&1 || { tail -40 gpurun_out/$TAG/rccl_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/rccl_tests.log
for n in 2 4; do
  HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python -u tools/bench_tpch.py --gpus $n --sf-per-gpu $((10 / n)) --steps 2 --warmup 1 > gpurun_out/$TAG/tpch_${n}rank.log 2>&1 || { tail -20 gpurun_out/$TAG/tpch_${n}rank.log; exit 1; }
  grep '^{' gpurun_out/$TAG/tpch_${n}rank.log | cut -c1-300
done
HPCJOIN_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --inner 2e8 --outer 2e8 --steps 3 --warmup 1 > gpurun_out/$TAG/bench_2rank.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_2rank.log; exit 1; }
grep '^{' gpurun_out/$TAG/bench_2rank.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["topology"]["rccl_transports"], d["shuffle_path"]["ms_per_step"], d["correct"])'
HPCJOIN_SHARE_GPU=1 timeout -k 10 500 python -u tools/bench_skew.py --gpus 8 --inner 1e8 --outer 4e8 --configs zipf_both --assign lpt,round_robin --split on,off > gpurun_out/$TAG/skew_8rank.jsonl 2>&1 || { tail -20 gpurun_out/$TAG/skew_8rank.jsonl; exit 1; }
grep '^{' gpurun_out/$TAG/skew_8rank.jsonl | cut -c1-200
echo done
