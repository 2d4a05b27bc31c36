#!/bin/bash
# round 6: packed multi-tenant curve K = 1 / 2 / 4 / 8 with the round-6 kernels
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 4 8; do
  timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pack_$k.json 2>>gpurun_out/pack.err || exit $?
done
grep -ho '"value": [0-9.]*' gpurun_out/pack_*.json
