#!/bin/bash
# DP-path numerics (world-1 RCCL / xGMI tests, fused-vs-unfused) + DP world-1 benches + 1-GPU bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dp_overlap.py tests/test_gpu_sync_bn.py tests/test_hip_step.py -m gpu > gpurun_out/dp_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dp_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/dp_pytest.log | head -80; exit $rc; }
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/dp_bench.json 2> gpurun_out/dp_bench.err || { tail -20 gpurun_out/dp_bench.err; exit 4; }
cat gpurun_out/dp_bench.json
for s in allreduce lowrank; do
  timeout -k 10 300 python scripts/bench_dp1.py --strategy $s --steps 3000 --warmup 300 > gpurun_out/dp_dp1_$s.json 2> gpurun_out/dp_dp1_$s.err || { tail -20 gpurun_out/dp_dp1_$s.err; exit 5; }
  cat gpurun_out/dp_dp1_$s.json
done
