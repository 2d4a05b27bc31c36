#!/bin/bash
# Quick check: HIP step numerics, per-launch times, default bench (2 runs).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_step.py tests/test_multitenant.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/q_tests.log | head -20; exit $rc; }
timeout -k 10 200 python scripts/microbench.py > gpurun_out/q_mb.txt 2>&1 || { tail -20 gpurun_out/q_mb.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/q_mb.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/q_bench_$i.json 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('gpurun_out/q_bench_$i.json'));print('bench', d['ms_per_step'], d['value'])"
done
