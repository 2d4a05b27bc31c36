#!/bin/bash
# Multi-process xGMI / async-PS tests on their own, then the driver's GPU suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4c_ps.log 2>&1
rc=$?; echo "xgmi rc=$rc"; grep -E "passed|failed" gpurun_out/r4c_ps.log | tail -3
[ $rc -ne 0 ] && { grep -E "AssertionError|RuntimeError|timed out" gpurun_out/r4c_ps.log | head -20; exit $rc; }
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4c_pytest.log | tail -3
[ $rc -ne 0 ] && { grep -B2 -A40 "FAILED\|Error" gpurun_out/r4c_pytest.log | tail -60; exit $rc; }
exit 0
