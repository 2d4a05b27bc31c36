#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py tests/test_deterministic.py -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/ab_pytest.log | head -60; exit $rc; }
for r in 1 2 3; do timeout -k 10 200 python bench.py --steps 3000 --warmup 300 | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])'; done
timeout -k 10 200 python scripts/microbench.py --reps 200 > gpurun_out/ab_mb.txt 2>&1; grep -v amdgpu gpurun_out/ab_mb.txt | tail -14
