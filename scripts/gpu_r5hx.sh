#!/bin/bash
# Round 5: the update body's weight-gradient A operands read in one LDS batch.  Numerics,
# the carried segment's stamps, the carrying launch, bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5hx_t.txt 2>&1 || { tail -30 gpurun_out/r5hx_t.txt; exit 3; }
tail -1 gpurun_out/r5hx_t.txt
MB_HF=1 MB_HF_ONLY=1 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5hx_1.txt 2>&1 || { tail -5 gpurun_out/r5hx_1.txt; exit 4; }
grep -E "HF:|carried|blocks \[" gpurun_out/r5hx_1.txt
MB_HF=1 MB_EDGES=828,1808 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5hx_a.txt 2>&1 || { tail -5 gpurun_out/r5hx_a.txt; exit 4; }
grep -E "HF:|life|blocks \[" gpurun_out/r5hx_a.txt
for r in 1 2; do
  a=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  b=$(timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
  echo "20/5 $a 2000/200 $b"
done
