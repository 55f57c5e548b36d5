#!/bin/bash
# Bitmap slice walks: per slice (0), flat (1), chained cross-slice pipeline (2),
# at 1B and 125M, alternated twice; walk tests first.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-ch}
timeout -k 10 300 python -u -m pytest tests/test_bitmap_plans.py -x -q -m gpu -k "walk or split or tiny" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
for size in 1e9 1.25e8; do
  for f in 0 1 2; do
    L=gpurun_out/${TAG}_${size}_${f}_${rep}.log
    HPCJOIN_BM_FLAT=$f timeout -k 10 200 python bench.py --inner $size --outer $size --steps 20 --warmup 3 --general off > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'flat', sys.argv[3], d['ms_per_step'], d['phases_ms']['dev_build_probe_ms'], d['correct'])" $L $size $f
  done
done
done
echo done
