#!/bin/bash
# Round-2 iteration: HIP step numerics tests, bench, kernel profile.  Every GPU step is
# time-limited; stop at the first failure.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
K=${1:-"hip_step"}
timeout -k 10 600 python -u -m pytest tests/test_hip_step.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hip.log 2>&1
rc=$?; tail -15 gpurun_out/t_hip.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r2" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 300 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r2.txt" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_r2.txt"; exit 5; }
cd "$GRAFT_REPO_ROOT" && python scripts/prof_summary.py gpurun_out/prof_r2 --steps 322 > gpurun_out/prof_r2.md && cat gpurun_out/prof_r2.md
