#!/bin/bash
# Round 5: the pair forward's load batch without whole batches past the weights / x tile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5fw_t.txt 2>&1 || { tail -30 gpurun_out/r5fw_t.txt; exit 3; }
tail -1 gpurun_out/r5fw_t.txt
MB_CP=1 MB_CP_BLOCKS=0,1,350,699 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5fw_mb.txt 2>&1 || { tail -5 gpurun_out/r5fw_mb.txt; exit 4; }
grep -E "conv_pair|sum of" gpurun_out/r5fw_mb.txt
for r in 1 2; do
  a=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  b=$(timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  echo "20/5 $a 2000/200 $b"
done
