#!/bin/bash
# Driver's exact GPU-suite command, then smoke, bench and a rocprofv3 kernel trace of the step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 900 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/r3c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Fatal|Error" gpurun_out/r3c_pytest.log | tail -8
[ $rc -ne 0 ] && { grep -B2 -A30 "FAILED\|Error\|csa-test" gpurun_out/r3c_pytest.log | tail -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.txt 2>&1 || { tail -20 gpurun_out/r3c_smoke.txt; exit 3; }
tail -1 gpurun_out/r3c_smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || { tail -20 gpurun_out/r3c_bench.err; exit 4; }
cat gpurun_out/r3c_bench.json
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/r3c_bench2000.json 2>> gpurun_out/r3c_bench.err || exit 5
cat gpurun_out/r3c_bench2000.json
rm -rf $R/gpurun_out/trace; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace --steps 1100 > gpurun_out/r3c_trace.md && cat gpurun_out/r3c_trace.md
