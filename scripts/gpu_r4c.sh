#!/bin/bash
# xGMI ps step with 2 processes on one GPU (diagnostics), then the remaining GPU tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
true
rc=0
[ $rc -ne 0 ] && { grep -E "RuntimeError|Error|timed out" gpurun_out/r4c_ps.log | head -20; exit $rc; }
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4c_pytest.log | tail -3
[ $rc -ne 0 ] && { grep -B2 -A40 "FAILED\|Error" gpurun_out/r4c_pytest.log | tail -60; exit $rc; }
exit 0
