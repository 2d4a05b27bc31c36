#!/bin/bash
# Phase stamps of the conv-pair / head / dense-update / optimizer kernels (one launch each).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_CP=1 MB_DU=1 MB_OPT=1 timeout -k 10 200 python scripts/microbench.py > gpurun_out/stamps.txt 2>&1 || { tail -20 gpurun_out/stamps.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/stamps.txt | grep -v "^ *[0-9] csa_[a-z_0-9]* *[0-9.]* us$"
