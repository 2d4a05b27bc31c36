#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in 200 350 700; do
  echo "== CSA_WGRAD_TARGET=$t"
  CSA_WGRAD_TARGET=$t timeout -k 10 300 python scripts/microbench.py > gpurun_out/mb_$t.log 2>&1 || { tail -5 gpurun_out/mb_$t.log; exit 3; }
  grep -E "conv_wgrad|optimizer|graph step" gpurun_out/mb_$t.log
done
