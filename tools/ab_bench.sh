#!/bin/bash
# Same-box A/B of bench.py variants (HPCJOIN_<FIELD>=value sets per run):
#   tools/ab_bench.sh TAG "general|head" "NET_THREADS=512" "LOCAL_GEOMETRY=1" ...
# An empty string runs the defaults.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=$1; MODE=$2; shift 2; mkdir -p gpurun_out/$TAG
G=off; [ "$MODE" = general ] && G=only
i=0
for v in "$@"; do
  i=$((i+1))
  env $(for kv in $v; do echo HPCJOIN_$kv; done) timeout -k 10 200 python -u bench.py --general $G --steps 10 --warmup 2 > gpurun_out/$TAG/ab_${MODE}_$i.log 2>&1 || { tail -20 gpurun_out/$TAG/ab_${MODE}_$i.log; exit 1; }
  echo "[$MODE $v] $(tail -1 gpurun_out/$TAG/ab_${MODE}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], d["correct"], p["dev_network_ms"], p["dev_local_partition_ms"], p["dev_build_probe_ms"])')"
done
