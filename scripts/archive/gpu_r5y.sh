#!/bin/bash
# Round 5: default multi-step graph size 32 — the GPU tests that replay groups, then the
# packed curve K = 1 / 2 / 4 / 8 at k = 32 and k = 8.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_multitenant.py tests/test_hip_step.py tests/test_gpu_platform.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5y_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5y_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 32 8; do for j in 1 2 4 8; do
  CSA_GRAPH_STEPS=$k timeout -k 10 150 python3 bench.py --jobs $j --steps 1600 --warmup 160 > gpurun_out/r5y_k${k}_j$j.json 2>> gpurun_out/r5y.err || exit 3
  echo "k=$k jobs=$j $(grep -o '"value": [0-9.]*' gpurun_out/r5y_k${k}_j$j.json)"
done; done
