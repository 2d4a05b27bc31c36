#!/bin/bash
# DP program on one GPU (world-1 RCCL group) per strategy + packed-host admission stall.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 > gpurun_out/da_bench.json 2> gpurun_out/da_bench.err || { tail -20 gpurun_out/da_bench.err; exit 4; }
cat gpurun_out/da_bench.json
for s in lowrank allreduce; do
  timeout -k 10 300 python scripts/bench_dp1.py --strategy $s --steps 3000 --warmup 300 > gpurun_out/da_dp1_$s.json 2> gpurun_out/da_dp1_$s.err || { tail -20 gpurun_out/da_dp1_$s.err; exit 5; }
  cat gpurun_out/da_dp1_$s.json
done
timeout -k 10 400 python scripts/bench_admission.py --jobs 4 --reps 3 > gpurun_out/da_admission.txt 2> gpurun_out/da_admission.err || { tail -20 gpurun_out/da_admission.err; exit 6; }
cat gpurun_out/da_admission.txt
