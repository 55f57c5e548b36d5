#!/bin/bash
# A/B of an env switch on the 1B x 1B headline bench (general path off): VAR=name, values in VALS.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2; do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --general off --steps 10 --warmup 2 > gpurun_out/abh_${v}.log 2>&1 || { tail -5 gpurun_out/abh_${v}.log; exit 1; }
  echo "$VAR=$v $(tail -1 gpurun_out/abh_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], p["dev_network_ms"], p["dev_build_probe_ms"], d["correct"])')"
done; done
