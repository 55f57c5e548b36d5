#!/bin/bash
# PMC passes over the 1B x 1B headline join (one counter group per run).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-pmc}; shift; BARGS="$@"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/${TAG}_$name -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 1 --general off $BARGS > $R/gpurun_out/${TAG}_$name.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_$name.log; return 1; }
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD && echo pmc done
