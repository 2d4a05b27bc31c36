#!/bin/bash
# GPU round check: @gpu tests, smoke, bench, rocprofv3 kernel stats, per-kernel microbench.
# Every GPU step is time-limited; the script stops at the first crash / timeout.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -30 gpurun_out/gpu_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 3; }
tail -2 gpurun_out/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 4; }
cat gpurun_out/bench_default.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hip" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 300 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_hip.txt" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_hip.txt"; exit 5; }
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/microbench.py > gpurun_out/micro.txt 2>&1 || { tail -20 gpurun_out/micro.txt; exit 6; }
tail -20 gpurun_out/micro.txt
exit $rc
