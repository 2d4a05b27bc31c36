#!/bin/bash
# Round 5: longer multi-step graphs — packed K = 4 / 8 and one job at k = 64 / 128 / 256.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 64 128 256; do for j in 1 4 8; do
  CSA_GRAPH_STEPS=$k timeout -k 10 150 python3 bench.py --jobs $j --steps 2048 --warmup 256 > gpurun_out/r5z_k${k}_j$j.json 2>> gpurun_out/r5z.err || exit 3
  echo "k=$k jobs=$j $(grep -o '"value": [0-9.]*' gpurun_out/r5z_k${k}_j$j.json)"
done; done
