#!/bin/bash
# Closing run: the whole-repo GPU check, a kernel trace of the step, in-graph workgroup
# stamps of one step (graph_life) and the carried-segment stamps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
rm -rf gpurun_out/final_tr
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/final_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1) || exit 6
python3 scripts/step_timeline.py $(find gpurun_out/final_tr -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 3 > gpurun_out/final_timeline.txt
cat gpurun_out/final_timeline.txt
MB_HF=1 MB_HF_ONLY=1 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/final_mb.txt 2>&1 || { tail -5 gpurun_out/final_mb.txt; exit 7; }
grep -E "HF:|carried" gpurun_out/final_mb.txt
timeout -k 10 180 python3 scripts/mb/graph_life.py --reps 2 > gpurun_out/final_glife.txt 2>&1 || { tail -5 gpurun_out/final_glife.txt; exit 8; }
head -14 gpurun_out/final_glife.txt
