#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_distributed.py -k "one_sided or rccl_multiprocess or in_process or hot_partition" > gpurun_out/onesided_pytest.log 2>&1 || { tail -40 gpurun_out/onesided_pytest.log; exit 1; }
tail -3 gpurun_out/onesided_pytest.log
