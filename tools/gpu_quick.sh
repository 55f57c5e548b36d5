#!/bin/bash
# Focused GPU check: selected tests -> smoke -> 1B bench (JSON) -> rocprofv3 kernel stats.
#   tools/gpu_quick.sh TAG "pytest selection" [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-quick}; SEL=${2:-tests/test_bitmap_plans.py}; shift 2; BARGS="$@"
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread $SEL -m gpu > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 $BARGS --json-out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); g=d.get('general_path') or {}; print(d['ms_per_step'], d['value'], d['correct'], d['first_join_ms'], d['config']['plan'], '| general', g.get('ms_per_step'), g.get('value'), g.get('correct'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 $BARGS > $R/gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_prof.log; exit 1; }
echo profiled
