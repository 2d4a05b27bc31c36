#!/bin/bash
# round 6: the pair backward's in-LDS GEMMs in masked 8-step groups — numerics, phases
# (MB_HF stamps), in-graph lives, 1-GPU A/B vs ab/r6d (HEAD)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py tests/test_gpu_health.py > gpurun_out/t_g8.log 2>&1 || { tail -30 gpurun_out/t_g8.log; exit 3; }
tail -1 gpurun_out/t_g8.log
for v in r6d new; do
  if [ $v = r6d ]; then export CSA_KERNEL_LIB=ab/r6d/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
  MB_HF=1 MB_CP_BLOCKS=0,350 $T 180 python scripts/microbench.py > gpurun_out/mbhf_g8_$v.txt 2>&1 || exit $?
  grep -E "HF:|block 0:|block 350:" gpurun_out/mbhf_g8_$v.txt
done
unset CSA_KERNEL_LIB
$T 180 python scripts/mb/graph_life.py --reps 1 > gpurun_out/glife_g8.txt 2>&1 || exit $?
grep -E "span|carrier" gpurun_out/glife_g8.txt
for r in 1 2 3; do
  for v in r6d new; do
    if [ $v = r6d ]; then export CSA_KERNEL_LIB=ab/r6d/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
for v in r6d new; do for n in 2000 20; do echo -n "$v $n: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_${n}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done; done
