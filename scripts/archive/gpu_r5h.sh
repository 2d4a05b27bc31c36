#!/bin/bash
# Round 5: packed K = 8 at k = 32 with 4 / 6 / 8 hardware queues per process.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for q in 4 6 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python3 bench.py --jobs 8 --steps 2048 --warmup 256 > gpurun_out/r5h_q$q.json 2>> gpurun_out/r5h.err || exit 3
  echo "hwq=$q jobs=8 $(grep -o '"value": [0-9.]*' gpurun_out/r5h_q$q.json)"
done
