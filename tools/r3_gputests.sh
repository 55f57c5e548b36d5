#!/bin/bash
# Full GPU test suite + smoke, then the default bench.  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3t}; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1 || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["general_path"]; print("head", d["ms_per_step"], d["first_join_ms"], d["setup_ms"], d["correct"], "general", g.get("ms_per_step"), g.get("first_join_ms"), g.get("correct"))'
