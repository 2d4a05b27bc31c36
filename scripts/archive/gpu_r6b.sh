#!/bin/bash
# round 6: carrier residency (LDS-DMA update body, 5 WG/CU) — numerics, then same-box A/B
# against ab/r6base (HEAD before the change), the watchdog probe and the new device tests
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T 200 python scripts/mb/watchdog_probe.py > gpurun_out/wd_probe.jsonl 2>gpurun_out/wd_probe.err || exit $?
$T 900 $PYT tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_health.py > gpurun_out/t_step.log 2>&1 || exit $?
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export CSA_KERNEL_LIB=ab/r6base/libcsa_kernels.so; else unset CSA_KERNEL_LIB; fi
    $T 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_${v}_20_$r.json 2>>gpurun_out/ab.err || exit $?
    $T 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/ab_${v}_2000_$r.json 2>>gpurun_out/ab.err || exit $?
  done
done
unset CSA_KERNEL_LIB
$T 900 $PYT tests/test_gpu_dp_overlap.py > gpurun_out/t_dp.log 2>&1 || exit $?
$T 900 $PYT tests/test_gpu_xgmi.py -k production > gpurun_out/t_prod.log 2>&1 || exit $?
