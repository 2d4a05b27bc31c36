#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dp_overlap.py tests/test_gpu_sync_bn.py tests/test_hip_step.py -m gpu > gpurun_out/dpt_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/dpt_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED" gpurun_out/dpt_pytest.log | head -80; exit $rc; }
for s in allreduce ps lowrank; do timeout -k 10 300 python scripts/bench_dp1.py --strategy $s --steps 3000 --warmup 300 2>/dev/null | tail -1; done
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 2>/dev/null | tail -1 | cut -c1-200
