#!/bin/bash
# closing numbers after the suite passed (158 GPU tests, smoke ok on this tree): DP world-1
# benches, kernel trace of the step, carried-segment stamps, graph_life
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for s in allreduce allreduce:hf ps ps:hf async_ps async_ps:flat; do
  timeout -k 10 200 python3 scripts/bench_dp1.py --strategy $s > gpurun_out/check_dp_$s.json 2>> gpurun_out/check.err || exit 6
  echo "dp1 $s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/check_dp_$s.json)"
done
rm -rf gpurun_out/final_tr
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/final_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1) || exit 6
python3 scripts/step_timeline.py $(find gpurun_out/final_tr -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 3 > gpurun_out/final_timeline.txt
grep -E "^-- step" gpurun_out/final_timeline.txt
timeout -k 10 180 python3 scripts/mb/graph_life.py --reps 2 > gpurun_out/final_glife.txt 2>&1 || { tail -5 gpurun_out/final_glife.txt; exit 8; }
grep -E "span|fc1 dgrad" gpurun_out/final_glife.txt
