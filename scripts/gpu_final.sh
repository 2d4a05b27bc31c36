#!/bin/bash
# Round-end rehearsal + packed curve.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_full.sh > gpurun_out/final_full.log 2>&1 || { tail -30 gpurun_out/final_full.log; exit 5; }
grep -E "passed|failed|smoke ok|\"metric\"" gpurun_out/final_full.log
bash scripts/gpu_pack5.sh
