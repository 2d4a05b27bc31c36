#!/bin/bash
# World-1 data-parallel programs (ps on the xGMI kernels / RCCL, allreduce) vs the 1-GPU program.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4t_1gpu.json 2>> gpurun_out/r4t.err || { tail -20 gpurun_out/r4t.err; exit 4; }
echo "1-GPU $(python3 -c "import json;d=json.load(open('gpurun_out/r4t_1gpu.json'));print(d['ms_per_step'])")"
for s in "ps 1" "ps 0" "allreduce 1" "allreduce 0"; do set -- $s
timeout -k 10 240 python scripts/bench_dp1.py --strategy $1 --xgmi $2 --steps 2000 --warmup 200 > gpurun_out/r4t_dp.json 2>> gpurun_out/r4t.err || { tail -20 gpurun_out/r4t.err; exit 5; }
echo "strategy=$1 xgmi=$2 $(tail -1 gpurun_out/r4t_dp.json | cut -c1-200)"
done
