#!/bin/bash
# Sweep one HPCJOIN_<FIELD> env override over the 1B x 1B bench:  tools/sweep_env.sh FIELD v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
F=$1; shift
for v in "$@"; do
  env HPCJOIN_$F=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/sweep_${F}_$v.log 2>&1 || { tail -5 gpurun_out/sweep_${F}_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${F}_$v.log').read().strip().splitlines()[-1]); print('$F=$v', d['value'], d['ms_per_step'], d['phases_ms'])"
done
