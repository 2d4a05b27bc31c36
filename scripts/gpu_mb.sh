#!/bin/bash
# Microbench: per-kernel isolated times + fused-kernel phase stamps (+ optional tests).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${1:-}" = "test" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_hip_step.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hip.log 2>&1
  rc=$?; tail -5 gpurun_out/t_hip.log; [ $rc -ne 0 ] && exit $rc
fi
MB_CP=1 MB_DU=1 timeout -k 10 300 python scripts/microbench.py --reps 200 > gpurun_out/micro.txt 2>&1 || { tail -20 gpurun_out/micro.txt; exit 6; }
cat gpurun_out/micro.txt | grep -v amdgpu.ids
