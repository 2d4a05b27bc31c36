#!/bin/bash
# Optimizer launch experiments: batch staging off, block caps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "CSA_STAGE_BATCH=1" "CSA_STAGE_BATCH=0" "CSA_OPT_MAX_BLOCKS=64" "CSA_OPT_MAX_BLOCKS=256"; do
  env $cfg timeout -k 10 120 python scripts/microbench.py --reps 200 > gpurun_out/optexp.txt 2>&1 || { tail -5 gpurun_out/optexp.txt; exit 3; }
  echo "$cfg: $(grep -E 'optimizer|head_part|conv_pair_fwd|graph step' gpurun_out/optexp.txt | awk '{print $2, $3}' | tr '\n' ' ')"
done
