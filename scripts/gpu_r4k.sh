#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_HF=1 timeout -k 10 200 python scripts/microbench.py --reps 200 > gpurun_out/r4k.txt 2>&1 || { tail -20 gpurun_out/r4k.txt; exit 6; }
grep -v amdgpu.ids gpurun_out/r4k.txt
