#!/bin/bash
# Standard GPU validation step: gpu tests -> smoke -> 1B bench -> micro-benchmarks.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; exit $rc; }
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 python tools/microbench.py all > gpurun_out/${TAG}_micro.log 2>&1 || { tail -20 gpurun_out/${TAG}_micro.log; exit 1; }
grep bench gpurun_out/${TAG}_micro.log
