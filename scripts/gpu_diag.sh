#!/bin/bash
# Diagnostics: DP tests, GEMM in-kernel stamps (WG 0) + one PMC pass over the step kernels.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp_overlap.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/dp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/dp_tests.log; [ $rc -gt 1 ] && exit $rc
MB_GEMM=1 timeout -k 10 300 python scripts/microbench.py --reps 50 > gpurun_out/micro_stamps.txt 2>&1 || { tail -20 gpurun_out/micro_stamps.txt; exit 3; }
grep stamps gpurun_out/micro_stamps.txt
bash scripts/gpu_pmc.sh pmc_a
exit $rc
