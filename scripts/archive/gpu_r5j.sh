#!/bin/bash
# Round 5: DP world-1 step timelines (allreduce on RCCL), per-bucket optimizer off / on.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for bo in 0 1; do
  cd /tmp && CSA_DP_BUCKET_OPT=$bo timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5j_$bo -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_dp1.py --strategy allreduce --xgmi 0 --steps 300 --warmup 50 > /dev/null 2>&1 || exit 3
  cd $GRAFT_REPO_ROOT; python3 scripts/step_timeline.py $(find gpurun_out/r5j_$bo -name "*kernel_trace.csv" | head -1) --skip 250 --steps 1 > gpurun_out/r5j_tl$bo.txt || exit 4
  echo "== bucket_opt=$bo"; cat gpurun_out/r5j_tl$bo.txt
done
