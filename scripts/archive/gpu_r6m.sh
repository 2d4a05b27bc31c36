#!/bin/bash
# round 6: VALU c1 recompute / dwA + bias sums (4 partial sums per thread) in the pair
# backward — numerics, phases (MB_HF stamps), A/B over CSA_CP_VALU = 0 / 1 / 3 and ab/r6c
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 600 $PYT tests/test_hip_step.py tests/test_deterministic.py > gpurun_out/t_step.log 2>&1 || exit $?
for v in 0 3; do
  CSA_CP_VALU=$v MB_HF=1 MB_CP_BLOCKS=0,350 $T 180 python scripts/microbench.py > gpurun_out/mbhf_v$v.txt 2>&1 || exit $?
done
for r in 1 2 3; do
  for v in r6c 0 1 3; do
    if [ $v = r6c ]; then export CSA_KERNEL_LIB=ab/r6c/libcsa_kernels.so; else unset CSA_KERNEL_LIB; export CSA_CP_VALU=$v; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
