#!/bin/bash
# Round 5: xGMI flag protocol (diagnostics, co-resident block cap, 2/4/8 ranks on one GPU),
# dedicated RCCL capture group, async_ps on the device at 2/4/8 ranks.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -v -p no:cacheprovider \
  --timeout 400 --timeout-method thread > gpurun_out/r5a.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5a.log | tail -30 | cut -c1-400; exit $rc
