#!/bin/bash
# Phase stamps of the conv pair / head kernels + the FUSED_DENSE=0 launch list for comparison.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_CP=1 MB_HEAD=1 timeout -k 10 200 python scripts/microbench.py > gpurun_out/stamps.txt 2>&1 || { tail -20 gpurun_out/stamps.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/stamps.txt
CSA_FUSED_DENSE=0 timeout -k 10 200 python scripts/microbench.py > gpurun_out/mb_nofuse.txt 2>&1 || { tail -20 gpurun_out/mb_nofuse.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/mb_nofuse.txt
