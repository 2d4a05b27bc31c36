#!/bin/bash
# Round 5: start / end of every workgroup in the carrying launch (pair | fc2 update |
# fc1 update | tail), to see which kind sits on the critical path; then the carried fc1
# update workgroups' phase stamps (fc1's segment alone).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp


MB_HF=1 MB_HF_ONLY=1 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5lf1.txt 2>&1 || { tail -5 gpurun_out/r5lf1.txt; exit 4; }
grep -E "HF:|life|blocks \[|p50|carried" gpurun_out/r5lf1.txt
