#!/bin/bash
# Phase stamps of every kernel family of the default step + isolated launch times.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_CP=1 MB_HEAD=1 MB_DU=1 MB_OPT=1 MB_DD=1 timeout -k 10 200 python scripts/microbench.py > gpurun_out/stamps.txt 2>&1 || { tail -20 gpurun_out/stamps.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/stamps.txt
