#!/bin/bash
# Fused row materialization: GPU tests, then SF100 fused vs unfused.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_join_engine.py tests/test_distributed.py -k "fused_row or materialize_split or tpch_late" \
  > gpurun_out/fused_pytest.log 2>&1 || { tail -30 gpurun_out/fused_pytest.log; exit 1; }
tail -3 gpurun_out/fused_pytest.log
timeout -k 10 300 python tools/bench_tpch.py --steps 3 --warmup 1 > gpurun_out/tpch_fused.log 2>&1 || { tail -5 gpurun_out/tpch_fused.log; exit 1; }
tail -1 gpurun_out/tpch_fused.log | cut -c1-900
timeout -k 10 300 python tools/bench_tpch.py --steps 3 --warmup 1 --unfused > gpurun_out/tpch_unfused.log 2>&1 || { tail -5 gpurun_out/tpch_unfused.log; exit 1; }
tail -1 gpurun_out/tpch_unfused.log | cut -c1-600
