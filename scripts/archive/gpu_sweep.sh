#!/bin/bash
# Sweep an env knob over values on the default bench (one box session).
# usage: bash scripts/gpu_sweep.sh VAR v1 v2 ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$1; shift
for val in "$@"; do
  env $V=$val timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/sweep_${V}_${val}.json 2>/dev/null || exit 3
  echo "$V=$val $(python -c "import json;d=json.load(open('gpurun_out/sweep_${V}_${val}.json'));print(d['ms_per_step'],d['value'])")"
done
