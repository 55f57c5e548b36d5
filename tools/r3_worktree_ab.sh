#!/bin/bash
# Same-box A/B of this tree against git worktrees (built in-tree, given as
# arguments): headline and general path, alternating twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out/wt
run() { (cd $1 && timeout -k 10 300 python -u bench.py --general $3 --steps 8 --warmup 2 > $R/gpurun_out/wt/$2.log 2>&1) || return 1
  echo "$2 $(tail -1 gpurun_out/wt/$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], d["correct"], p["dev_network_ms"], p["dev_local_partition_ms"], p["dev_build_probe_ms"])')"; }
for rep in 1 2; do
  run $R head_h$rep off || exit 1
  for w in "$@"; do run $R/$w ${w}_h$rep off || exit 1; done
  run $R head_g$rep only || exit 1
  for w in "$@"; do run $R/$w ${w}_g$rep only || exit 1; done
done
