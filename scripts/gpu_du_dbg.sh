#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in ${DBGS:-0}; do
  echo "== CSA_DU_DBG=$d"
  CSA_DU_DBG=$d MB_DU=1 timeout -k 10 120 python scripts/microbench.py --reps 100 2>&1 | grep -vE "amdgpu.ids" || exit 1
done
