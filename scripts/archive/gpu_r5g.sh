#!/bin/bash
# Round 5: how the packed profile's kernels scale with batch (a stand-in for grouping G
# jobs into one launch): per-kernel us at B = 50 / 100 / 200 / 400.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 50 100 200 400; do
  timeout -k 10 200 python3 scripts/microbench.py --packed --batch $b --reps 100 > gpurun_out/r5g_b$b.txt 2>&1 || { tail -5 gpurun_out/r5g_b$b.txt; exit 3; }
  echo "== B=$b"; cat gpurun_out/r5g_b$b.txt | tail -25
done
