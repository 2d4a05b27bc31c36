#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py -m gpu > gpurun_out/hs_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/hs_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/hs_pytest.log | head -60; exit $rc; }
exit 0
