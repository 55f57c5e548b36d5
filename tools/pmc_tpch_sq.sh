#!/bin/bash
# SQ counters (wait / busy / LDS instructions / bank conflicts) of the SF100 TPC-H-like bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $R/gpurun_out/tpch_sq -o run --output-format csv -- python $R/tools/bench_tpch.py --steps 1 --warmup 0 > $R/gpurun_out/tpch_sq.log 2>&1 && echo done
