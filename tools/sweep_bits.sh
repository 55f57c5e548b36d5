#!/bin/bash
# Sweep the (network, local) radix split on the 1B x 1B headline config.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for nb in "9 9" "10 8" "8 10" "11 7"; do
  set -- $nb
  HPCJOIN_NETWORK_BITS=$1 HPCJOIN_LOCAL_BITS=$2 timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/sweep_$1_$2.log 2>&1 || { tail -5 gpurun_out/sweep_$1_$2.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sweep_$1_$2.log') if l.startswith('{')][-1]); print($1,$2,d['value'],d['ms_per_step'],d['correct'],d['phases_ms'])"
done
