#!/bin/bash
# rocprofv3 kernel traces of the DP program on one GPU (world-1 RCCL group), per strategy.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for s in allreduce lowrank; do
  rm -rf $R/gpurun_out/trace_dp_$s; cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_dp_$s -o run -- python3 $R/scripts/bench_dp1.py --strategy $s --steps 1000 --warmup 100 > $R/gpurun_out/trace_dp_$s.log 2>&1 || { tail -5 $R/gpurun_out/trace_dp_$s.log; exit 3; }
  cd $R && python3 scripts/prof_summary.py gpurun_out/trace_dp_$s --steps 1100 --top 30 > gpurun_out/trace_dp_$s.md && cat gpurun_out/trace_dp_$s.md
done
