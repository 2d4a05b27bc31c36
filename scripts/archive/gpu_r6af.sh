#!/bin/bash
# round 6: split-K width of the register-direct dense forwards (target waves per launch)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for t in 2048 1536 2560 3072; do
    CSA_DD_TARGET=$t timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/dd_${t}_2000_$r.json 2>>gpurun_out/dd.err || exit $?
    CSA_DD_TARGET=$t timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/dd_${t}_20_$r.json 2>>gpurun_out/dd.err || exit $?
  done
done
for t in 2048 1536 2560 3072; do for n in 2000 20; do echo -n "$t $n: "; for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/dd_${t}_${n}_$r.json | cut -d' ' -f2 | tr '\n' ' '; done; echo; done; done
