#!/bin/bash
# Fused dense backward + update (tile design): numerics, per-launch times, A/B bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CSA_FUSED_DENSE=1 timeout -k 10 400 python -u -m pytest tests/test_hip_step.py -x -q --timeout 120 --timeout-method thread > gpurun_out/du_tests.log 2>&1
rc=$?; tail -3 gpurun_out/du_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/du_tests.log | head -20; exit $rc; }
CSA_FUSED_DENSE=1 MB_DU=1 timeout -k 10 200 python scripts/microbench.py > gpurun_out/du_mb.txt 2>&1 || { tail -20 gpurun_out/du_mb.txt; exit 3; }
cat gpurun_out/du_mb.txt
bash scripts/gpu_ab.sh CSA_FUSED_DENSE 0 1
