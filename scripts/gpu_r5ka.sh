#!/bin/bash
# Round 5: does the kernel-argument placement matter (HIP_FORCE_DEV_KERNARG)?  The carried
# update body reads its segment descriptor (DUSegs, ~1.2 KB) from the kernarg segment.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 0; do
  HIP_FORCE_DEV_KERNARG=$k MB_HF=1 MB_HF_ONLY=1 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5ka_$k.txt 2>&1 || { tail -5 gpurun_out/r5ka_$k.txt; exit 4; }
  echo "devkernarg=$k"; grep -E "HF:|carried" gpurun_out/r5ka_$k.txt
done
for r in 1 2; do
  for k in 0 1; do
    a=$(HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "devkernarg=$k 20/5 $a 2000/200 $b"
  done
done
