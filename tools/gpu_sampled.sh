#!/bin/bash
# Sampled group totals (netSampledTotals): full GPU suite, 1B and 125M joins
# (bitmap plan) and the 1B general path, then a kernel trace at 125M.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-samp}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_1b.log 2>&1 || { tail -20 gpurun_out/${TAG}_1b.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['general_path']; print('1b', d['ms_per_step'], d['correct'], d['engine']['network_fallbacks'], 'general', g['ms_per_step'], g['correct'])" gpurun_out/${TAG}_1b.log
timeout -k 10 200 python bench.py --inner 1.25e8 --outer 1.25e8 --steps 20 --warmup 3 --general off > gpurun_out/${TAG}_125m.log 2>&1 || { tail -20 gpurun_out/${TAG}_125m.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('125m', d['ms_per_step'], d['correct'], d['engine']['network_fallbacks'])" gpurun_out/${TAG}_125m.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p125m -o run --output-format csv -- python $R/bench.py --inner 1.25e8 --outer 1.25e8 --steps 20 --warmup 3 --general off > $R/gpurun_out/${TAG}_p125m.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_p125m.log; exit 1; }
echo done
