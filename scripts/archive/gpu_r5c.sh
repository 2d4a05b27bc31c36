#!/bin/bash
# Round 5: the world-2 flag loss (scripts/gpu_r5b.sh reproduced it in every variant within
# 26 steps) with the failing call's per-block record kept; world 2 and 3, 200 steps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp CSA_XGMI_TIMEOUT_S=3
out=gpurun_out/r5c.jsonl; : > $out
for w in 2 3 2; do
  timeout -k 10 200 python3 scripts/xgmi_stress.py --world $w --steps 200 >> $out 2>> gpurun_out/r5c.err
  rc=$?; echo "w=$w rc=$rc"
  [ $rc -gt 1 ] && { tail -5 gpurun_out/r5c.err; exit $rc; }
done
exit 0
