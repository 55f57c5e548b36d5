#!/bin/bash
# Bitmap kernels: flat vs per-slice claim-slice walk and 1024 / 256 threads.
# Bitmap GPU tests, then 1B and 125M (one N = 8 rank's share) joins, and the
# 8-rank in-process rehearsal (replicated-bitmap build + probe kernels).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-bmwalk}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "bitmap or Bitmap" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for size in 1e9 1.25e8; do
  for v in "auto auto" "1024 0" "1024 1" "256 0" "256 1"; do
    set -- $v
    env_nth=""; env_flat=""
    [ "$1" != auto ] && export HPCJOIN_BM_NTH=$1 || unset HPCJOIN_BM_NTH
    [ "$2" != auto ] && export HPCJOIN_BM_FLAT=$2 || unset HPCJOIN_BM_FLAT
    L=gpurun_out/${TAG}_${size}_$1_$2.log
    timeout -k 10 200 python bench.py --inner $size --outer $size --steps 20 --warmup 3 --general off > $L 2>&1 || { tail -20 $L; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['phases_ms']['dev_build_probe_ms'], d['correct'])" $L $size "$v"
  done
done
unset HPCJOIN_BM_NTH HPCJOIN_BM_FLAT
timeout -k 10 200 python tools/rehearse_inprocess.py --ranks 8 --size 1e9 > gpurun_out/${TAG}_inproc8.log 2>&1 || { tail -20 gpurun_out/${TAG}_inproc8.log; exit 1; }
grep -o '"join_ms": [0-9.]*' gpurun_out/${TAG}_inproc8.log | head -1
HPCJOIN_BM_FLAT=0 timeout -k 10 200 python tools/rehearse_inprocess.py --ranks 8 --size 1e9 > gpurun_out/${TAG}_inproc8_noflat.log 2>&1 || { tail -20 gpurun_out/${TAG}_inproc8_noflat.log; exit 1; }
grep -o '"join_ms": [0-9.]*' gpurun_out/${TAG}_inproc8_noflat.log | head -1
echo done
