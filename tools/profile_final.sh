#!/bin/bash
# End-of-session evidence: kernel stats of the 1B headline + general path,
# then PMC passes (FETCH, WRITE, SQ) over the headline join.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
TAG=${1:-fin}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_stats -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/${TAG}_stats.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_stats.log; exit 1; }
cd $R && bash tools/pmc_headline.sh ${TAG}_pmc
