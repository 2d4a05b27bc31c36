#!/bin/bash
# Round 5: the carrying launch with wide (1024-thread) vs narrow (128-column) fc1 update
# blocks: pair alone / updates alone / fused, and the update blocks' start spread.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in 1 0; do
  CSA_DU_WIDE=$w MB_HF=1 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5wd_$w.txt 2>&1 || { tail -5 gpurun_out/r5wd_$w.txt; exit 4; }
  echo "wide=$w"; grep -E "HF:|segment" gpurun_out/r5wd_$w.txt
done
