#!/bin/bash
# Round-4: bench A/B (CSA_HFUSE 0/1, 2000 steps) + driver-shaped bench, then numerics
# (test_hip_step, DP overlap / ps, xGMI) and a kernel trace of the default program.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for i in 1 2; do for h in 0 1; do
CSA_HFUSE=$h timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4b_bench_h${h}_$i.json 2> gpurun_out/r4b_bench.err || { tail -20 gpurun_out/r4b_bench.err; exit 4; }
echo "hfuse=$h $(python3 -c "import json;d=json.load(open('gpurun_out/r4b_bench_h${h}_$i.json'));print(d['ms_per_step'], d['value'])")"
done; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r4b_bench20.json 2>> gpurun_out/r4b_bench.err || exit 5
cat gpurun_out/r4b_bench20.json
timeout -k 10 700 python3 -u -m pytest tests/test_hip_step.py tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4b_pytest.log | tail -3
[ $rc -ne 0 ] && { grep -B2 -A40 "FAILED\|Error" gpurun_out/r4b_pytest.log | tail -80; exit $rc; }
rm -rf $R/gpurun_out/trace; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace --steps 1100 > gpurun_out/r4b_trace.md && cat gpurun_out/r4b_trace.md
