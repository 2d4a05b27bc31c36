#!/bin/bash
# Kernel-numerics GPU tests + bench + isolated per-launch timings with pair phase stamps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_serving.py -m gpu > gpurun_out/q_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/q_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/q_pytest.log | head -80; exit $rc; }
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -20 gpurun_out/q_bench.err; exit 4; }
cat gpurun_out/q_bench.json
timeout -k 10 200 env MB_CP=1 python scripts/microbench.py --reps 200 > gpurun_out/q_mb.txt 2>&1 || { tail -20 gpurun_out/q_mb.txt; exit 5; }
cat gpurun_out/q_mb.txt
