#!/bin/bash
# Round 3: new GPU tests (packed multi-step / re-pack, DP lowrank fused update), DP world-1
# bench vs the 1-GPU bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_gpu_platform.py -k "packed" tests/test_gpu_dp_overlap.py > gpurun_out/r3a_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|stall|passed|failed" gpurun_out/r3a_tests.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { tail -20 gpurun_out/r3a_bench.err; exit 4; }
cat gpurun_out/r3a_bench.json
for s in lowrank allreduce; do
  timeout -k 10 300 python scripts/bench_dp1.py --strategy $s > gpurun_out/r3a_dp1_$s.json 2> gpurun_out/r3a_dp1_$s.err || { tail -20 gpurun_out/r3a_dp1_$s.err; exit 5; }
  cat gpurun_out/r3a_dp1_$s.json
done
