#!/bin/bash
# Sampled N > 1 network pass: in-process GPU tests, then the RCCL worker
# (2 and 4 processes sharing the GPU).  TAG = output dir.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3p}; mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py -k "sampled" > gpurun_out/$TAG/sampled_tests.log 2>&1 || { tail -60 gpurun_out/$TAG/sampled_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/$TAG/sampled_tests.log | tail -14
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_distributed.py -k "rccl_multiprocess and (2 or 4)" > gpurun_out/$TAG/rccl_tests.log 2>&1 || { tail -60 gpurun_out/$TAG/rccl_tests.log; exit 1; }
tail -3 gpurun_out/$TAG/rccl_tests.log
