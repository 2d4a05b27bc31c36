#!/bin/bash
# A/B an env toggle on the default bench in one box session: alternate A,B,A,B.
# usage: bash scripts/gpu_ab.sh VAR valA valB
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$1; A=$2; B=$3
for i in 1 2; do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/ab_${V}_${val}_$i.json 2>/dev/null || exit 3
    echo "$V=$val run$i $(python -c "import json;d=json.load(open('gpurun_out/ab_${V}_${val}_$i.json'));print(d['ms_per_step'],d['value'])")"
  done
done
