#!/bin/bash
# round 6: packed K = 2 / 4 / 8 — packed launch shapes vs the one-job shapes (both with hfuse)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for k in 2 4 8; do
    timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pks_p_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
    CSA_PACKED_PROFILE=0 timeout -k 10 300 python bench.py --jobs $k --steps 1024 --warmup 128 > gpurun_out/pks_s_${k}_$r.json 2>>gpurun_out/pack.err || exit $?
  done
done
for f in gpurun_out/pks_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
