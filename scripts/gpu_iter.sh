#!/bin/bash
# One iteration of the kernel loop: numerics tests, bench, per-kernel microbench
# (+ head phase stamps).  Stops at the first failing GPU step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_hip_step.py -x -q -m gpu > gpurun_out/hip_tests.log 2>&1
rc=$?; tail -15 gpurun_out/hip_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -20 gpurun_out/bench_iter.err; exit 3; }
cat gpurun_out/bench_iter.json
timeout -k 10 300 python scripts/microbench.py > gpurun_out/micro.log 2>&1 || { tail -20 gpurun_out/micro.log; exit 4; }
cat gpurun_out/micro.log | tail -40
exit $rc
