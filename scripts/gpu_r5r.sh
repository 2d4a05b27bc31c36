#!/bin/bash
# Round 5: horizontal-fusion microbenchmark — pair backward alone, the deferred dense
# updates alone, both in one launch, per-block phase stamps of the update segments.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_HF=1 timeout -k 10 200 python3 scripts/microbench.py --reps 200 > gpurun_out/r5r.txt 2>&1 || { tail -20 gpurun_out/r5r.txt; exit 3; }
grep -E "HF:|block 0|segment" gpurun_out/r5r.txt
