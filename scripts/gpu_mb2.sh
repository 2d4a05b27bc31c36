#!/bin/bash
# Isolated launches: default vs deterministic (exclusive stripes: no atomic contention), optimizer stamps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 env MB_OPT=1 MB_DU=1 python scripts/microbench.py --reps 200 > gpurun_out/mb2_default.txt 2>&1 || { tail -20 gpurun_out/mb2_default.txt; exit 1; }
timeout -k 10 200 env CSA_DETERMINISTIC=1 python scripts/microbench.py --reps 200 > gpurun_out/mb2_det.txt 2>&1 || { tail -20 gpurun_out/mb2_det.txt; exit 2; }
grep -v amdgpu.ids gpurun_out/mb2_default.txt; echo ---det---; grep -v amdgpu.ids gpurun_out/mb2_det.txt
