#!/bin/bash
# Tests + per-launch times + A/B of the fc1 decomposition (1024-thread row groups vs
# 128-column blocks with the partial hand-off).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_DU=1 bash scripts/gpu_quick.sh || exit $?
bash scripts/gpu_ab3.sh CSA_DU_WIDE_MIN_GROUPS=128 CSA_DU_WIDE_MIN_GROUPS=100000
