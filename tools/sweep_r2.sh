#!/bin/bash
# Headline variants (1B x 1B, general path off): scatter tile and bitmap unroll.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-sweep}
for v in "NET_IPT=8 BM_U=4" "NET_IPT=16 BM_U=4" "NET_IPT=8 BM_U=8" "NET_IPT=16 BM_U=8"; do
  set -- $v
  env HPCJOIN_$1 HPCJOIN_$2 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --general off > gpurun_out/${TAG}_${1}_${2}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${1}_${2}.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/${TAG}_${1}_${2}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["correct"], d["phases_ms"]["dev_network_ms"], d["phases_ms"]["dev_build_probe_ms"])')"
done
