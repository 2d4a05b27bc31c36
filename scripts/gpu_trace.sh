#!/bin/bash
# rocprofv3 kernel trace of the default captured step (bench, 1000 steps).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/trace
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 3; }
cd $R && grep '"metric"' gpurun_out/trace.log | tail -1
