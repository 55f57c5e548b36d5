#!/bin/bash
# General path (key-only words): key-only GPU tests, then the 1B x 1B sparse-key
# bench and its kernel stats.  TAG names the output directory.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3g}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bitmap_plans.py tests/test_join_engine.py -k "sparse64 or key_only or oracle" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u bench.py --general only --steps 10 --warmup 2 > gpurun_out/$TAG/bench.log 2>&1 || { tail -5 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("ms_per_step"), d.get("value"), d.get("correct"), d.get("phases_ms"))'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/stats -o run --output-format csv -- python $R/bench.py --general only --steps 3 --warmup 1 > $R/gpurun_out/$TAG/stats.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/stats.log; exit 1; }
echo done
