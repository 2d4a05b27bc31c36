#!/bin/bash
# round 6: the production DP programs at world 4 (opt-in case: four ranks time-slicing the
# box's one GPU), once, with a long per-spawn bound
set -o pipefail
mkdir -p gpurun_out
CSA_TEST_WORLD4=1 CSA_TEST_PROD_TIMEOUT=1000 timeout -k 10 1150 python -u -m pytest -x -v --timeout 1100 --timeout-method thread tests/test_gpu_xgmi.py -k "production and 4" > gpurun_out/t_prod4.log 2>&1
rc=$?; tail -15 gpurun_out/t_prod4.log; exit $rc
