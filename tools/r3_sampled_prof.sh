#!/bin/bash
# Kernel trace of a 2-process shared-GPU bench.py (headline, shuffle_path and
# general_path at 2e8 x 2e8): each rank under its own rocprofv3 (bash starts
# both, nothing GPU-initialised execs).  The sampled N > 1 network pass shows
# netSampledHistogramKernel and no full-input netHistogramKernel on the
# shuffle and general paths.  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3q}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 HPCJOIN_SHARE_GPU=1
cd /tmp && export TMPDIR=/tmp
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_r$r -o r$r --output-format csv -- python3 -u $R/bench.py --gpus 2 --inner 2e8 --outer 2e8 --steps 3 --warmup 1 > $OUT/bench_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -30 $OUT/bench_r0.log; tail -10 $OUT/bench_r1.log; exit 1; }
grep '^{' $OUT/bench_r0.log | python3 -c '
import json,sys; d=json.loads(sys.stdin.read())
for k in ("shuffle_path","general_path"):
    x=d[k]; print(k, x["ms_per_step"], x["correct"], x["sampled_network"], x["network_fallbacks"], x["phases_ms"])
print("head", d["ms_per_step"], d["correct"])'
find $OUT/prof_r0 -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 -c '
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n=r["Name"]
    if "Histogram" in n or "Scatter" in n or "wire" in n or "segCopy" in n or "ChunkGroup" in n:
        print(r["Calls"], round(float(r["TotalDurationNs"])/1e6,2), "ms", n[:90])' {}
