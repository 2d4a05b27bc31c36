#!/bin/bash
# Round 5: kernel trace of the data-parallel ":hf" program at world 1 with the dense update
# carried by the pair forward (profiles/r5_dp_trace.md).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5t2_dp -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_dp1.py --strategy allreduce:hf --xgmi 0 --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python3 scripts/step_timeline.py $(find gpurun_out/r5t2_dp -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 2
