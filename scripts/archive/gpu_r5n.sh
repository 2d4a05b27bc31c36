#!/bin/bash
# Round 5: packed jobs vs HIP hardware queues per process (K branches of one graph map onto
# at most GPU_MAX_HW_QUEUES queues).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for q in 4 8 16; do for k in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --jobs $k --pack graph --steps 1000 --warmup 100 > gpurun_out/r5n_${k}_$q.json 2>> gpurun_out/r5n.err || exit 3
  echo "K=$k hwq=$q $(grep -o '"value": [0-9.]*' gpurun_out/r5n_${k}_$q.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5n_${k}_$q.json)"
done; done
