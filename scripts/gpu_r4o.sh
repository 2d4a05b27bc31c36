#!/bin/bash
# xGMI multi-process tests in suite order (pooled peer buffers).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4o.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r4o.log | tail -25
[ $rc -ne 0 ] && { grep -E "AssertionError|RuntimeError|timed out" gpurun_out/r4o.log | head -10; exit $rc; }
exit 0
