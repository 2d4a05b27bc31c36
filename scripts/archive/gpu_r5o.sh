#!/bin/bash
# Round 5: async_ps step time on the device transport — world 1 (bench_dp1) and 2 ranks
# sharing the one GPU (xgmi_stress) — beside the synchronous programs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/bench_dp1.py --strategy async_ps --xgmi 0 --steps 2000 --warmup 200 > gpurun_out/r5o_aps1.json 2>> gpurun_out/r5o.err || exit 3
echo "async_ps world 1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5o_aps1.json)"
CSA_XGMI_BLOCKS=256 timeout -k 10 200 python3 scripts/xgmi_stress.py --world 2 --steps 300 --strategy async_ps > gpurun_out/r5o_aps2.json 2>> gpurun_out/r5o.err; rc=$?
echo "async_ps world 2 (one GPU): rc=$rc $(cut -c1-600 gpurun_out/r5o_aps2.json)"
