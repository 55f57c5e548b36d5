R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum -d $R/gpurun_out/tpch_fetch -o run --output-format csv -- python $R/tools/bench_tpch.py --steps 1 --warmup 0 > $R/gpurun_out/tpch_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_MISS_sum -d $R/gpurun_out/tpch_write -o run --output-format csv -- python $R/tools/bench_tpch.py --steps 1 --warmup 0 > $R/gpurun_out/tpch_write.log 2>&1 && echo done
