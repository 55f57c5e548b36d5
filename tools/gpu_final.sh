#!/bin/bash
# End-of-session check: full GPU suite, smoke, default bench, 4B x 4B capacity run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], d['correct'], 'general', d['general_path']['ms_per_step'], d['general_path']['correct'])" gpurun_out/${TAG}_bench.log
timeout -k 10 500 python bench.py --inner 4e9 --outer 4e9 --steps 3 --warmup 1 --general off > gpurun_out/${TAG}_4b.log 2>&1 || { tail -20 gpurun_out/${TAG}_4b.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('4b', d['ms_per_step'], d['value'], d['correct'], d['config']['plan'], d['engine']['workspace_peak_GB'])" gpurun_out/${TAG}_4b.log
echo done
