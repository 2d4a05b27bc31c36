#!/bin/bash
# Driver's exact GPU-suite command, then smoke, bench and the DP world-1 benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/r3b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Fatal|Error" gpurun_out/r3b_pytest.log | tail -8; [ $rc -ne 0 ] && { grep -B2 -A20 "FAILED\|Error" gpurun_out/r3b_pytest.log | head -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.txt 2>&1 || { tail -20 gpurun_out/r3b_smoke.txt; exit 3; }
tail -1 gpurun_out/r3b_smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || { tail -20 gpurun_out/r3b_bench.err; exit 4; }
cat gpurun_out/r3b_bench.json
for s in lowrank allreduce; do
  timeout -k 10 300 python scripts/bench_dp1.py --strategy $s > gpurun_out/r3b_dp1_$s.json 2> gpurun_out/r3b_dp1_$s.err || { tail -20 gpurun_out/r3b_dp1_$s.err; exit 5; }
  cat gpurun_out/r3b_dp1_$s.json
done
