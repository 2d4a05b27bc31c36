#!/bin/bash
# Iteration loop: HIP step numerics tests, bench (default), isolated launch list + graph step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_step.py ${TESTS_EXTRA} > gpurun_out/iter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/iter_tests.log; [ $rc -ne 0 ] && { grep -B5 -A25 "Error\|FAILED" gpurun_out/iter_tests.log | head -80; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || { tail -20 gpurun_out/iter_bench.err; exit 4; }
cat gpurun_out/iter_bench.json
timeout -k 10 200 python scripts/microbench.py > gpurun_out/iter_mb.txt 2>&1 || { tail -20 gpurun_out/iter_mb.txt; exit 5; }
grep -v amdgpu.ids gpurun_out/iter_mb.txt
