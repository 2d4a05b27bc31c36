#!/bin/bash
# round 6: packed K = 4 / 8 with the one-GPU fused program per job (CSA_PACKED_HFUSE=1) vs default
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for k in 4 8; do
    timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/packd_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
    CSA_PACKED_HFUSE=1 timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/packh_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
  done
done
for f in gpurun_out/packd_* gpurun_out/packh_*; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
