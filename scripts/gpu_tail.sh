#!/bin/bash
# Step-tail (no optimizer launch) numerics + A/B bench + microbench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py tests/test_deterministic.py -m gpu > gpurun_out/t_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/t_pytest.log | head -80; exit $rc; }
for r in 1 2 3; do
  for v in 1 0; do
    ms=$(env CSA_STEP_TAIL=$v timeout -k 10 120 python bench.py --steps 3000 --warmup 300 | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') || exit 1
    echo "CSA_STEP_TAIL=$v $ms" | tee -a gpurun_out/ab_tail.txt
  done
done
timeout -k 10 200 env MB_CP=1 python scripts/microbench.py --reps 200 > gpurun_out/t_mb.txt 2>&1 || { tail -20 gpurun_out/t_mb.txt; exit 5; }
cat gpurun_out/t_mb.txt
