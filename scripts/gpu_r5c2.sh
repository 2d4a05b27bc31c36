#!/bin/bash
# Round 5: deferred dense update carried by the next step's pair forward (DP all-reduce
# programs): the DP / sync-BN / xGMI GPU tests, then world-1 timings with and without it.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_sync_bn.py tests/test_gpu_xgmi.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r5c2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5c2_tests.log; [ $rc -ne 0 ] && exit $rc
for c in 1 0; do for s in allreduce:hf allreduce; do
  CSA_DP_CARRY=$c timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $s > gpurun_out/r5c2_${c}_$s.json 2>> gpurun_out/r5c2.err || exit 3
  echo "carry=$c $s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5c2_${c}_$s.json)"
done; done
