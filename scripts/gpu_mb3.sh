#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py -m gpu -k "optimizers or fused_update or staged or step_matches" > gpurun_out/mb3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/mb3_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/mb3_pytest.log | head -60; exit $rc; }
timeout -k 10 200 env MB_OPT=1 MB_DU=1 python scripts/microbench.py --reps 200 > gpurun_out/mb3.txt 2>&1 || { tail -20 gpurun_out/mb3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/mb3.txt
for r in 1 2; do timeout -k 10 200 python bench.py --steps 3000 --warmup 300 | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])'; done
