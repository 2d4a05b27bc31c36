#!/bin/bash
# Whole-repo GPU check: the GPU suite, smoke(), the driver's bench shape, DP world-1 programs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/check_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/check_tests.log | tail -5 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check_smoke.txt 2>&1 || { tail -20 gpurun_out/check_smoke.txt; exit 3; }
tail -1 gpurun_out/check_smoke.txt
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/check_b20.json 2>> gpurun_out/check.err || exit 4
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/check_b2000.json 2>> gpurun_out/check.err || exit 5
echo "bench 20/5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/check_b20.json); 2000/200 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/check_b2000.json)"
for s in allreduce allreduce:hf ps ps:hf async_ps async_ps:flat; do
  timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $s > gpurun_out/check_dp_$s.json 2>> gpurun_out/check.err || exit 6
  echo "dp1 $s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/check_dp_$s.json)"
done
