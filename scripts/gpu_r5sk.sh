#!/bin/bash
# Round 5: the pair backward's prologue no longer issues load batches that lie wholly past
# an operand (index tables, weight panels, x tile, route rows).  Numerics, stamps, bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5sk_t.txt 2>&1 || { tail -30 gpurun_out/r5sk_t.txt; exit 3; }
tail -1 gpurun_out/r5sk_t.txt
MB_HF=1 MB_CP_BLOCKS=1,350,699 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5sk_mb.txt 2>&1 || { tail -5 gpurun_out/r5sk_mb.txt; exit 4; }
grep -E "HF:|pair alone block|updates block" gpurun_out/r5sk_mb.txt
for r in 1 2 3; do
  a=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  b=$(timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  echo "20/5 $a 2000/200 $b"
done
