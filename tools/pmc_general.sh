#!/bin/bash
# SQ counters of the general path (key-only words) bench: wait / busy / LDS / bank conflicts per kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/general_sq -o run --output-format csv -- python $R/bench.py --general only --steps 1 --warmup 0 > $R/gpurun_out/general_sq.log 2>&1 && echo done
