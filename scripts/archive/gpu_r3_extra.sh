#!/bin/bash
# Round-3 evidence refresh: serving latency, packed curve K = 2 / 4 / 8, preprocessing throughput.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_inference.py > gpurun_out/x_infer.txt 2>&1 || { tail -20 gpurun_out/x_infer.txt; exit 1; }
grep -v amdgpu gpurun_out/x_infer.txt | tail -6
for K in 2 4 8; do
  timeout -k 10 300 python bench.py --jobs $K --pack graph --steps 2000 --warmup 200 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$K', d['value'], d['ms_per_step'])" || exit 2
done
timeout -k 10 300 python scripts/bench_preprocess.py > gpurun_out/x_pre.txt 2>&1 || { tail -20 gpurun_out/x_pre.txt; exit 3; }
grep -v amdgpu gpurun_out/x_pre.txt | tail -20
