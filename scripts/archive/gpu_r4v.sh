#!/bin/bash
# ps on RCCL without bucket overlap: DP tests + world-1 timing.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dp_overlap.py tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r4v.log 2>&1 || { grep -E "passed|failed|Error" gpurun_out/r4v.log | tail -8 | cut -c1-300; exit 3; }
grep -E "passed|failed" gpurun_out/r4v.log | tail -1
timeout -k 10 240 python scripts/bench_dp1.py --strategy ps --xgmi 0 --steps 2000 --warmup 200 > gpurun_out/r4v_dp.json 2>> gpurun_out/r4v.err || { tail -20 gpurun_out/r4v.err; exit 5; }
echo "ps rccl $(tail -1 gpurun_out/r4v_dp.json | cut -c1-90)"
