#!/bin/bash
# Packed-host admission / retirement stall + the packed GPU tests and the GC regression test.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_platform.py tests/test_gpu_dp_overlap.py tests/test_multitenant.py -m gpu > gpurun_out/adm_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/adm_pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED" gpurun_out/adm_pytest.log | head -80; exit $rc; }
timeout -k 10 400 python scripts/bench_admission.py --jobs 4 --reps 3 > gpurun_out/adm.txt 2> gpurun_out/adm.err || { tail -20 gpurun_out/adm.err; exit 6; }
cat gpurun_out/adm.txt
timeout -k 10 300 python bench.py --jobs 4 --pack graph --steps 2000 --warmup 200 > gpurun_out/adm_pack4.json 2> gpurun_out/adm_pack4.err || { tail -20 gpurun_out/adm_pack4.err; exit 7; }
cat gpurun_out/adm_pack4.json
