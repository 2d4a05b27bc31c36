#!/bin/bash
# Round 5: the driver's bench shape (20 / 5) as one 20-step graph replay vs the k = 8
# groups (8 + 8 + 4), three alternating rounds; and 2000 / 200 at k = 8 / 16 / 32.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for one in 1 0; do
    CSA_BENCH_ONE_GRAPH=$one timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5x_$one.json 2>> gpurun_out/r5x.err || exit 3
    echo "20/5 one_graph=$one $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5x_$one.json)"
  done
done
for k in 8 16 32; do
  CSA_GRAPH_STEPS=$k timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 > gpurun_out/r5x_k$k.json 2>> gpurun_out/r5x.err || exit 4
  echo "2000/200 k=$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5x_k$k.json)"
done
