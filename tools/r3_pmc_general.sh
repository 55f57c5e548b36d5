#!/bin/bash
# SQ counters of the general path (key-only words), one join; TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${1:-r3p}; mkdir -p $R/gpurun_out/$TAG; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/$TAG/sq -o run --output-format csv -- python $R/bench.py --general only --steps 1 --warmup 0 > $R/gpurun_out/$TAG/sq.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -d $R/gpurun_out/$TAG/sq2 -o run --output-format csv -- python $R/bench.py --general only --steps 1 --warmup 0 > $R/gpurun_out/$TAG/sq2.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/sq2.log; exit 1; }
echo pmc done
