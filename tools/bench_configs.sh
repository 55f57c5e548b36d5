#!/bin/bash
# All BASELINE.json configs that fit one MI355X, one JSON line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-cfg}
run() { local name=$1; shift; timeout -k 10 400 "$@" > gpurun_out/${TAG}_${name}.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/${TAG}_${name}.log; return 1; }; echo "$name $(tail -1 gpurun_out/${TAG}_${name}.log | cut -c1-400)"; }
run 1b python bench.py --steps 10 --warmup 2 && \
run 128m python bench.py --inner 1.28e8 --outer 1.28e8 --steps 20 --warmup 3 --general off && \
run zipf_1b_4b python bench.py --dist zipf --theta 0.75 --outer 4e9 --steps 5 --warmup 2 --general off && \
run uniform_1b_4b python bench.py --dist uniform --outer 4e9 --steps 5 --warmup 2 --general off && \
run tpch_sf100 python tools/bench_tpch.py && \
run pinned_1b python bench.py --input pinned --steps 3 --warmup 1 --general off
