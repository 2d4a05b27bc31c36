#!/bin/bash
# A/B a knob on the bench: ab_env.sh VAR "valA valB" [rounds]  (alternating runs, ms/step)
set -o pipefail
var=$1; vals=$2; rounds=${3:-3}
mkdir -p gpurun_out
for r in $(seq $rounds); do
  for v in $vals; do
    ms=$(env $var=$v timeout -k 10 120 python bench.py --steps 3000 --warmup 300 | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') || exit 1
    echo "$var=$v $ms" | tee -a gpurun_out/ab.txt
  done
done
