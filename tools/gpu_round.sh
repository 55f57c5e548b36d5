#!/bin/bash
# One GPU validation round: gpu tests -> 1B bench -> rocprofv3 kernel stats of the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-round}
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
echo profiled
