#!/bin/bash
# Kernel trace of the Zipf-both general path (sparse keys) at 1e9 x 4e9 with
# counted spans: per-kernel time of the build/probe after the first join
# switched every partition to counted tables (keyCount 9).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3cntp}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u $R/tools/bench_skew.py --inner 1e9 --outer 4e9 --steps 2 --warmup 1 --configs zipf_both_sparse > $OUT/skew.jsonl 2> $OUT/skew.err || { tail -5 $OUT/skew.err; exit 1; }
cut -c1-200 $OUT/skew.jsonl
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-5
