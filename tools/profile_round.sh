#!/bin/bash
# rocprofv3 kernel stats of the 1B x 1B bench + PMC counters (separate pass).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_stats -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_stats.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_stats.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $R/gpurun_out/${TAG}_sq -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/${TAG}_sq.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_sq.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum -d $R/gpurun_out/${TAG}_fetch -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/${TAG}_fetch.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_MISS_sum -d $R/gpurun_out/${TAG}_write -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/${TAG}_write.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_write.log; exit 1; }
echo done
