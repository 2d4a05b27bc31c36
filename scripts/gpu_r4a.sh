#!/bin/bash
# Round-4 baseline: driver GPU suite, smoke, driver-shaped bench (20/5) vs long bench
# (2000/200), and a rocprofv3 kernel trace of the step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4_pytest.log | tail -3
[ $rc -ne 0 ] && { grep -B2 -A30 "FAILED\|Error" gpurun_out/r4_pytest.log | tail -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.txt 2>&1 || { tail -20 gpurun_out/r4_smoke.txt; exit 3; }
tail -1 gpurun_out/r4_smoke.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench20_$i.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 4; }
cat gpurun_out/r4_bench20_$i.json
done
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4_bench2000.json 2>> gpurun_out/r4_bench.err || exit 5
cat gpurun_out/r4_bench2000.json
rm -rf $R/gpurun_out/trace; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace --steps 1100 > gpurun_out/r4a_trace.md && cat gpurun_out/r4a_trace.md
