#!/bin/bash
# A/B/C of env settings on the default bench: each "VAR=val[,VAR=val]" config twice.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "$@"; do
    env ${cfg//,/ } timeout -k 10 300 python bench.py --steps 3000 --warmup 300 > gpurun_out/ab3.json 2>/dev/null || exit 3
    echo "$cfg run$i $(python -c "import json;d=json.load(open('gpurun_out/ab3.json'));print(d['ms_per_step'],d['value'])")"
  done
done
