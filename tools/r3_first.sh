#!/bin/bash
# Cold first join of the headline: phase trace, allocation trace and a kernel
# trace (first join vs the steady ones).  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3f}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
HPCJOIN_TRACE_FIRST=1 HPCJOIN_TRACE_ALLOC=1 timeout -k 10 200 python -u bench.py --general off --steps 3 --warmup 1 > $OUT/first.log 2>&1 || { tail -20 $OUT/first.log; exit 1; }
grep -v '^{"metric' $OUT/first.log | tail -20
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python3 $R/bench.py --general off --steps 3 --warmup 1 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# joins start at the first sampled-totals kernel of the bitmap plan
starts = [i for i, r in enumerate(rows) if "SampledTotals" in r["Kernel_Name"] or "netSampledTotals" in r["Kernel_Name"]]
print("join starts at dispatch", starts[:6], "of", len(rows))
for j, s in enumerate(starts[:3]):
    e = starts[j + 1] if j + 1 < len(starts) else len(rows)
    t0 = int(rows[s]["Start_Timestamp"])
    print(f"join {j}: span {(int(rows[e-1]['End_Timestamp']) - t0)/1e6:.3f} ms")
    for r in rows[s:e]:
        print(f"   +{(int(r['Start_Timestamp'])-t0)/1e6:8.3f} {(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6:7.3f} {r['Kernel_Name'][:70]}")
PY
