#!/bin/bash
# Round 5 (late): the packed curve K = 1 / 2 / 4 / 8 (32-step graphs) after the pair-backward
# changes (BatchNorm tables, dead load batches, update-body LDS batch).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for j in 1 2 4 8; do
  timeout -k 10 150 python3 bench.py --jobs $j --steps 2048 --warmup 256 > gpurun_out/r5pk_j$j.json 2>> gpurun_out/r5pk.err || exit 3
  echo "jobs=$j $(grep -o '"value": [0-9.]*' gpurun_out/r5pk_j$j.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5pk_j$j.json)"
done
