#!/bin/bash
# Round 5: streaming optimizer kernel (no folds) — DP numerics + world-1 timings + timeline.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_hip_step.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r5l.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/r5l.log | tail -8 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for st in allreduce allreduce:hf ps ps:hf; do
  timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $st --xgmi 0 --steps 2000 --warmup 200 > gpurun_out/r5l_${st/:/_}.json 2>> gpurun_out/r5l.err || exit 4
  echo "$st $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5l_${st/:/_}.json)"
done
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5l_bench.json 2>> gpurun_out/r5l.err || exit 5
echo "1-GPU $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5l_bench.json)"
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5l_tr -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_dp1.py --strategy allreduce:hf --xgmi 0 --steps 300 --warmup 50 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT; python3 scripts/step_timeline.py $(find gpurun_out/r5l_tr -name "*kernel_trace.csv" | head -1) --skip 250 --steps 1
