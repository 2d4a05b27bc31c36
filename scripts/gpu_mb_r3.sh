#!/bin/bash
# Isolated per-launch timings + conv-pair phase stamps (block 0) for the default step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 env MB_CP=1 python scripts/microbench.py --reps 200 > gpurun_out/mb_r3.txt 2>&1 || { tail -20 gpurun_out/mb_r3.txt; exit 1; }
timeout -k 10 200 env CSA_PAIR_BN_TAB=0 MB_CP=1 python scripts/microbench.py --reps 200 > gpurun_out/mb_r3_notab.txt 2>&1 || { tail -20 gpurun_out/mb_r3_notab.txt; exit 1; }
timeout -k 10 200 env CSA_CP_MFMA=1 MB_CP=1 python scripts/microbench.py --reps 200 > gpurun_out/mb_r3_mfma.txt 2>&1 || { tail -20 gpurun_out/mb_r3_mfma.txt; exit 1; }
cat gpurun_out/mb_r3.txt gpurun_out/mb_r3_notab.txt gpurun_out/mb_r3_mfma.txt
