#!/bin/bash
# World-1 DP on RCCL: bucketed overlap on / off.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for s in "ps 0" "ps 1" "allreduce 0" "allreduce 1"; do set -- $s
CSA_DP_OVERLAP=$2 timeout -k 10 240 python scripts/bench_dp1.py --strategy $1 --xgmi 0 --steps 2000 --warmup 200 > gpurun_out/r4u_dp.json 2>> gpurun_out/r4u.err || { tail -20 gpurun_out/r4u.err; exit 5; }
echo "strategy=$1 overlap=$2 $(tail -1 gpurun_out/r4u_dp.json | cut -c1-90)"
done
