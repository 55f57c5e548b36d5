R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=r3x; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels.py tests/test_bitmap_plans.py > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 300 python -u bench.py --dist uniform --outer 4e9 --steps 5 --warmup 2 --general off > gpurun_out/$TAG/u14.log 2>&1 || exit 1
echo "uniform_1b_4b $(tail -1 gpurun_out/$TAG/u14.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["correct"], d["phases_ms"])')"
timeout -k 10 600 python -u tools/bench_skew.py --configs zipf_both > gpurun_out/$TAG/skew.jsonl 2> gpurun_out/$TAG/skew.err || { tail -5 gpurun_out/$TAG/skew.err; exit 1; }
tail -1 gpurun_out/$TAG/skew.jsonl | cut -c1-200
bash tools/ab_bench.sh $TAG general "" "NET_IPT=17" "" "NET_IPT=17" || exit 1
