#!/bin/bash
# Spans of partitions with repeated keys on counted tables
# (bpKeyCountedSpansKernel): key-only GPU tests, the unique-key general path,
# and Zipf duplicates on both sides through the sparse key bijection (general
# path) at 1e8 x 4e8 (10 + 9 radix bits) and 1e9 x 4e9.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3cnt}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
show() { python -c 'import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["config"], d["ms_per_step"], d["matches"], d["expected_matches"], d["correct"], d["phases_ms"])' $1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bitmap_plans.py -k "key_only or quotient or sparse64 or device_layout or past_2g" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/ab_bench.sh $TAG general "" "" || exit 1
HPCJOIN_NETWORK_BITS=10 HPCJOIN_LOCAL_BITS=9 timeout -k 10 600 python -u tools/bench_skew.py --inner 1e8 --outer 4e8 --configs zipf_both_sparse,zipf_both > $OUT/skew_1e8_10_9.jsonl 2> $OUT/skew.err || { tail -5 $OUT/skew.err; exit 1; }
show $OUT/skew_1e8_10_9.jsonl
timeout -k 10 800 python -u tools/bench_skew.py --inner 1e9 --outer 4e9 --steps 2 --warmup 1 --configs zipf_both_sparse,zipf_both,uniform_sparse > $OUT/skew_1e9.jsonl 2> $OUT/skew9.err || { tail -5 $OUT/skew9.err; exit 1; }
show $OUT/skew_1e9.jsonl
