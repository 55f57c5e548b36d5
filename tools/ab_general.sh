#!/bin/bash
# Same-box A/B of general-path variants: HPCJOIN_<FIELD>=value sets per run
# (config_from_dict), e.g.  tools/ab_general.sh r3g "SPLIT_LOCAL=0 KEY_COUNT=6" "SPLIT_LOCAL=1 KEY_COUNT=7"
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=$1; shift; mkdir -p gpurun_out/$TAG
i=0
for v in "$@"; do
  i=$((i+1))
  env $(for kv in $v; do echo HPCJOIN_$kv; done) timeout -k 10 200 python -u bench.py --general only --steps 8 --warmup 2 > gpurun_out/$TAG/ab_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/ab_$i.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/$TAG/ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["correct"], d["phases_ms"]["dev_network_ms"], d["phases_ms"]["dev_local_partition_ms"], d["phases_ms"]["dev_build_probe_ms"])')"
done
