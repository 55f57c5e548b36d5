#!/bin/bash
# General path (random 63-bit keys) at one N = 8 rank's share, 125M x 125M:
# bench + kernel trace (fixed per-join costs).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-g125}
timeout -k 10 300 python bench.py --inner 1.25e8 --outer 1.25e8 --general only --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['correct'], d['phases_ms'])" gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_p -o run --output-format csv -- python $R/bench.py --inner 1.25e8 --outer 1.25e8 --general only --steps 10 --warmup 3 > $R/gpurun_out/${TAG}_p.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_p.log; exit 1; }
echo done
