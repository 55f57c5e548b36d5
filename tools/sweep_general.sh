#!/bin/bash
# General path (sparse 63-bit keys, key-only words) variants: build target / LDS table size.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-gsweep}
for v in ${VARIANTS:-"BUILD_TARGET=4096 R_CHUNK=0" "BUILD_TARGET=2048 R_CHUNK=2048" "BUILD_TARGET=8192 R_CHUNK=0"}; do
  set -- $v
  env HPCJOIN_$1 HPCJOIN_$2 timeout -k 10 200 python bench.py --steps 6 --warmup 1 --general only > gpurun_out/${TAG}_${1}_${2}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${1}_${2}.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/${TAG}_${1}_${2}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], d["value"], d["correct"], p["dev_network_ms"], p["dev_local_partition_ms"], p["dev_build_probe_ms"], d["config"]["plan"][:80])')"
done
