#!/bin/bash
# Round 5: the carrying launch WITH its tail (as in the step graph): every workgroup's
# start / end (pair | fc2 update | fc1 update | tail).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MB_HF=1 MB_TAIL=1 MB_EDGES=828,1808 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5tl.txt 2>&1 || { tail -5 gpurun_out/r5tl.txt; exit 4; }
grep -E "HF:|life|blocks \[|p50" gpurun_out/r5tl.txt
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5tl_t.txt 2>&1 || { tail -30 gpurun_out/r5tl_t.txt; exit 3; }
tail -1 gpurun_out/r5tl_t.txt
for r in 1 2; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    a=$(cd $d && timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(cd $d && timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "$v 20/5 $a 2000/200 $b"
  done
done
