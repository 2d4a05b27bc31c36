#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_platform.py tests/test_hip_step.py tests/test_gpu_dp_overlap.py -m gpu > gpurun_out/pk_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pk_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/pk_pytest.log | head -60; exit $rc; }
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/pk_bench.json 2>/dev/null || exit 4
cat gpurun_out/pk_bench.json
for K in 4 8; do
  timeout -k 10 300 python bench.py --jobs $K --pack graph --steps 2000 --warmup 200 > gpurun_out/pk_pack$K.json 2> gpurun_out/pk_err.log || { tail gpurun_out/pk_err.log; exit 7; }
  cat gpurun_out/pk_pack$K.json
done
timeout -k 10 400 python scripts/bench_admission.py --jobs 4 --reps 2 > gpurun_out/pk_adm.txt 2> gpurun_out/pk_adm.err || { tail -20 gpurun_out/pk_adm.err; exit 6; }
tail -1 gpurun_out/pk_adm.txt
