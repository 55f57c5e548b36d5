R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmc; cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || true
timeout -k 10 300 python $R/tools/microbench.py copy > $R/gpurun_out/pmc/copy.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $R/gpurun_out/pmc/sq -o run --output-format csv -- python $R/tools/microbench.py partition --iters 2 > $R/gpurun_out/pmc/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc/tcc -o run --output-format csv -- python $R/tools/microbench.py partition --iters 2 > $R/gpurun_out/pmc/tcc.log 2>&1
echo rc $?
