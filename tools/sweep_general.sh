#!/bin/bash
# General path (sparse 63-bit keys, key-only words) variants: build target / LDS table size.
#   VARIANTS="4096:0 2048:2048" tools/sweep_general.sh TAG   (build_target:r_chunk pairs)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-gsweep}
for v in ${VARIANTS:-4096:0 2048:2048 1024:1024}; do
  bt=${v%%:*}; rc=${v##*:}
  HPCJOIN_BUILD_TARGET=$bt HPCJOIN_R_CHUNK=$rc timeout -k 10 200 python bench.py --steps 6 --warmup 1 --general only > gpurun_out/${TAG}_${bt}_${rc}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${bt}_${rc}.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/${TAG}_${bt}_${rc}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_ms"]; print(d["ms_per_step"], d["value"], d["correct"], p["dev_network_ms"], p["dev_local_partition_ms"], p["dev_build_probe_ms"], d["config"]["plan"][:60])')"
done
