#!/bin/bash
# Packed K = 4 / 8 with fc1 as 1024-thread row groups (default) vs 128-column blocks.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for K in 4 8; do
  for v in 128 100000; do
    CSA_DU_WIDE_MIN_GROUPS=$v timeout -k 10 240 python bench.py --jobs $K --pack graph --steps 2000 --warmup 200 > gpurun_out/p3.json 2> gpurun_out/pack_err.log || exit 7
    python -c "import json; d=json.load(open('gpurun_out/p3.json')); print('K=$K wide_min=$v', d['value'], d['ms_per_step'])"
  done
done
