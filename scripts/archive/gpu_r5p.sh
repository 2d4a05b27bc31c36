#!/bin/bash
# Round 5: the pair forward's BatchNorm-apply workgroups (no bn_act_apply launch): numerics,
# A/B bench, kernel trace of the 1-GPU step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r5p.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/r5p.log | tail -8 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  CSA_FWD_APPLY=0 timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5p_b0_$i.json 2>> gpurun_out/r5p.err || exit 4
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5p_b1_$i.json 2>> gpurun_out/r5p.err || exit 5
  echo "apply=0 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5p_b0_$i.json)  apply=1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5p_b1_$i.json)"
done
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5p_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 500 --warmup 50 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT; python3 scripts/step_timeline.py $(find gpurun_out/r5p_tr -name "*kernel_trace.csv" | head -1) --skip 400 --steps 1
