#!/bin/bash
# Key-only count kernels: 4-slot (1 = default, 2) vs 2-slot buckets (6, 7):
# variant tests, then the 1B general path per variant (alternated twice).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-kc2}
timeout -k 10 300 python -u -m pytest tests/test_bitmap_plans.py -x -q -m gpu -k "key_only or sparse64" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for v in 1 6 7; do
    L=gpurun_out/${TAG}_v${v}_${rep}.log
    HPCJOIN_KCOUNT=$v timeout -k 10 200 python bench.py --general only --steps 10 --warmup 2 > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('v', sys.argv[2], d['ms_per_step'], d['phases_ms']['dev_build_probe_ms'], d['correct'])" $L $v
  done
done
echo done
