#!/bin/bash
# A/B of an env switch on the general-path bench: VAR=name, values in VALS.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --general only --steps 5 --warmup 1 > gpurun_out/ab_${v}.log 2>&1 || { tail -5 gpurun_out/ab_${v}.log; exit 1; }
  echo "$VAR=$v $(tail -1 gpurun_out/ab_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d.get("general_path") or d; p=g["phases_ms"]; print(g["ms_per_step"], p["dev_local_partition_ms"], p["dev_build_probe_ms"], g["correct"])')"
done; done
