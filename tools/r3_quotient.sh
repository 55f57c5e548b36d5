#!/bin/bash
# Quotient-table key-only count (keyCount 8): GPU tests, then a same-box A/B
# of the general path against the v2 span kernel (keyCount 7) and kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3k}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bitmap_plans.py -k "key_only or quotient or sparse64" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_general.sh $TAG "KEY_COUNT=8" "KEY_COUNT=7" "KEY_COUNT=8" "KEY_COUNT=7" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/bench.py --general only --steps 3 --warmup 1 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $OUT/stats -name "*kernel_stats.csv" | head -1) > $OUT/kernel_stats.md 2>&1; head -12 $OUT/kernel_stats.md
