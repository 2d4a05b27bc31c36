#!/bin/bash
# Round 5: per-phase s_memtime stamps of several pair-backward workgroups (not only block 0,
# which alone also does the BatchNorm running-statistic read-modify-write).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_HF=1 MB_CP_BLOCKS=0,1,100,350,600,699 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5bk.txt 2>&1 || { tail -5 gpurun_out/r5bk.txt; exit 3; }
grep -E "HF:|block" gpurun_out/r5bk.txt
