#!/bin/bash
# General path (key-only words): GPU tests, then the 1B x 1B sparse-key bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bitmap_plans.py tests/test_join_engine.py -k "sparse64 or key_only or oracle" > gpurun_out/general_pytest.log 2>&1 || { tail -30 gpurun_out/general_pytest.log; exit 1; }
tail -2 gpurun_out/general_pytest.log
timeout -k 10 300 python bench.py --general only --steps 5 --warmup 1 > gpurun_out/general_bench.log 2>&1 || { tail -5 gpurun_out/general_bench.log; exit 1; }
tail -1 gpurun_out/general_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d.get("general_path") or d; print(g.get("ms_per_step"), g.get("value"), g.get("correct"), g.get("phases_ms"))'
