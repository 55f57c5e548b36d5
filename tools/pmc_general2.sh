#!/bin/bash
# PMC passes over the general path (key-only words): SQ wait/busy/LDS and
# LDS-wait/VMEM-wait split, one pass each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-gpmc}
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/${TAG}_sq -o run --output-format csv -- python $R/bench.py --general only --steps 1 --warmup 0 > $R/gpurun_out/${TAG}_sq.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY -d $R/gpurun_out/${TAG}_wait -o run --output-format csv -- python $R/bench.py --general only --steps 1 --warmup 0 > $R/gpurun_out/${TAG}_wait.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_wait.log; exit 1; }
echo done
