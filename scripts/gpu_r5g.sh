#!/bin/bash
# Round 5: pair-backward tail, A/B against the optimizer launch (+ numerics).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_hip_step.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r5g.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/r5g.log | tail -8 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  CSA_PAIR_TAIL=0 timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5g_b0_$i.json 2>> gpurun_out/r5g.err || exit 4
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5g_b1_$i.json 2>> gpurun_out/r5g.err || exit 5
  echo "tail=0 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5g_b0_$i.json)  tail=1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5g_b1_$i.json)"
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5g_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/r5g_prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-8
