#!/bin/bash
# One iteration of the kernel loop: step numerics tests, bench, per-kernel microbench with
# GEMM stamps.  Stops at the first failing GPU step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_step.py tests/test_gpu_dp_overlap.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hip_tests.log 2>&1
rc=$?; tail -5 gpurun_out/hip_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -20 gpurun_out/bench_iter.err; exit 3; }
cat gpurun_out/bench_iter.json
MB_GEMM=1 timeout -k 10 300 python scripts/microbench.py --reps 100 > gpurun_out/micro.txt 2>&1 || { tail -20 gpurun_out/micro.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/micro.txt
exit $rc
