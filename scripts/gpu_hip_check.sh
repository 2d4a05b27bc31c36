#!/bin/bash
# HIP program: numerics tests vs torch, then bench (graph) and a kernel-trace profile.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_hip_step.py -x -q -m gpu > gpurun_out/hip_tests.log 2>&1
rc=$?
tail -30 gpurun_out/hip_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --backend hip --steps 2000 --warmup 200 > gpurun_out/bench_hip.json 2> gpurun_out/bench_hip.err || { cat gpurun_out/bench_hip.err | tail -20; exit 3; }
cat gpurun_out/bench_hip.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hip" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --backend hip --steps 300 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_hip.log" 2>&1
exit $rc
