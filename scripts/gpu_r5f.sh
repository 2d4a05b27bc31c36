#!/bin/bash
# Round 5: the pair-backward tail program (no optimizer launch): numerics + bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r5f.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/r5f.log | tail -8 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  CSA_PAIR_TAIL=0 timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5f_b0_$i.json 2>> gpurun_out/r5f.err || exit 4
  timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5f_b1_$i.json 2>> gpurun_out/r5f.err || exit 5
  echo "tail=0 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f_b0_$i.json)  tail=1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f_b1_$i.json)"
done
timeout -k 10 200 python3 bench.py > gpurun_out/r5f_default.json 2>> gpurun_out/r5f.err || exit 6
cut -c1-300 gpurun_out/r5f_default.json
