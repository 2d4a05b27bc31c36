#!/bin/bash
# Packed K = 8: kernel-shape knobs that trade one job's latency for CU-time.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "CSA_CP_PR=1" "CSA_CP_PR=2" "CSA_CP_PR=3" "CSA_OPT_MAX_BLOCKS=256" "CSA_STAGE_BATCH=0"; do
  env $cfg timeout -k 10 240 python bench.py --jobs 8 --pack graph --steps 2000 --warmup 200 > gpurun_out/p4.json 2> gpurun_out/pack_err.log || exit 7
  python -c "import json; d=json.load(open('gpurun_out/p4.json')); print('K=8 $cfg', d['value'], d['ms_per_step'])"
done
