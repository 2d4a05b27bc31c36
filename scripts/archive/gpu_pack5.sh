#!/bin/bash
# Packed curve (bench.py --jobs K builds its engines with the packed launch profile).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for K in 2 4 8; do
  timeout -k 10 240 python bench.py --jobs $K --pack graph --steps 2000 --warmup 200 > gpurun_out/p5_$K.json 2> gpurun_out/pack_err.log || exit 7
  python -c "import json; d=json.load(open('gpurun_out/p5_$K.json')); print('K=$K', d['value'], d['ms_per_step'], d['final_loss'])"
done
timeout -k 10 300 python -u -m pytest tests/test_multitenant.py tests/test_gpu_platform.py -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -2
