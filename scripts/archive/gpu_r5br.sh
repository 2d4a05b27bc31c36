#!/bin/bash
# Round 5: fc1's deferred update as a graph branch on a side stream (CSA_DENSE_BRANCH=1)
# instead of inside the pair backward — numerics with it on, then bench A/B and a trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CSA_DENSE_BRANCH=1 timeout -k 10 400 python3 -u -m pytest tests/test_hip_step.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5br_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5br_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for b in 0 1; do
  CSA_DENSE_BRANCH=$b timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5br_$b.json 2>> gpurun_out/r5br.err || exit 3
  CSA_DENSE_BRANCH=$b timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5br_l$b.json 2>> gpurun_out/r5br.err || exit 4
  echo "branch=$b 20/5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5br_$b.json) 2000/200 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5br_l$b.json)"
done; done
cd /tmp && CSA_DENSE_BRANCH=1 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5br_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python3 scripts/step_timeline.py $(find gpurun_out/r5br_tr -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 2
