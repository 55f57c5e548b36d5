#!/bin/bash
# Same-box A/B of the 1B x 4B uniform bitmap config: this tree vs the worktree(s) given as arguments.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/bisect
run() { (cd $1 && timeout -k 10 300 python -u bench.py --dist uniform --outer 4e9 --steps 5 --warmup 2 --general off > $R/gpurun_out/bisect/$2.log 2>&1) || return 1
  echo "$2 $(tail -1 gpurun_out/bisect/$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["correct"], d["phases_ms"]["dev_network_ms"], d["phases_ms"]["dev_build_probe_ms"])')"; }
for rep in 1 2; do
  run $R head$rep || exit 1
  for w in "$@"; do run $R/$w $w$rep || exit 1; done
done
