#!/bin/bash
# Round 5: DP program with per-bucket optimizer updates on the side stream + one-launch
# pair folds; world-1 A/B (allreduce / ps on RCCL and xGMI) + DP numerics + 1-GPU bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_hip_step.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r5i.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/r5i.log | tail -8 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for st in allreduce ps; do for x in 0 1; do for bo in 0 1; do
  CSA_DP_BUCKET_OPT=$bo timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $st --xgmi $x --steps 2000 --warmup 200 > gpurun_out/r5i_$st$x$bo.json 2>> gpurun_out/r5i.err || exit 4
  echo "$st xgmi=$x bucket_opt=$bo $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5i_$st$x$bo.json)"
done; done; done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5i_bench.json 2>> gpurun_out/r5i.err || exit 5
echo "1-GPU $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5i_bench.json)"
