#!/bin/bash
# Split bitmap pieces (21 fragment bits at N = 1): split tests + bitmap tests,
# then 3B x 3B (32-bit dense keys over a 2048-way digit) and the 1B headline.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-sp}
timeout -k 10 300 python -u -m pytest tests/test_bitmap_plans.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 400 python bench.py --inner 3e9 --outer 3e9 --steps 5 --warmup 2 --general off > gpurun_out/${TAG}_3b.log 2>&1 || { tail -20 gpurun_out/${TAG}_3b.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('3b', d['ms_per_step'], d['value'], d['correct'], d['config']['plan'], d['phases_ms'], d['engine']['workspace_peak_GB'])" gpurun_out/${TAG}_3b.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --general off > gpurun_out/${TAG}_1b.log 2>&1 || { tail -20 gpurun_out/${TAG}_1b.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('1b', d['ms_per_step'], d['value'], d['correct'])" gpurun_out/${TAG}_1b.log
echo done
