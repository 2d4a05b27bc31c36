#!/bin/bash
# Deterministic-mode lowerings first, then the multi-process xGMI / async-PS tests, then the suite.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_deterministic.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4e_det.log 2>&1
rc=$?; echo "det rc=$rc"; grep -E "passed|failed" gpurun_out/r4e_det.log | tail -3
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/r4e_det.log | tail -60; exit $rc; }
bash scripts/gpu_r4c.sh
