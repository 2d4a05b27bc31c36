#!/bin/bash
# Packed jobs: horizontal fusion / carrier / hardware-queue A/B and a kernel trace of the K = 4 pack.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
pk() {  # env-spec K
env $1 timeout -k 10 200 python bench.py --jobs $2 --pack graph --steps 2000 --warmup 200 > gpurun_out/r4g_p.json 2>> gpurun_out/r4g.err || { tail -20 gpurun_out/r4g.err; exit 4; }
echo "$1 K=$2 $(python3 -c "import json;d=json.load(open('gpurun_out/r4g_p.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2; do for k in 4 8; do
pk CSA_HFUSE=1 $k; pk CSA_HFUSE=0 $k; pk CSA_DU_CARRIER=opt $k
done; done
for q in 8 16; do pk GPU_MAX_HW_QUEUES=$q 8; done
rm -rf $R/gpurun_out/trace_pack; cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_pack -o run -- python3 $R/bench.py --jobs 4 --pack graph --steps 1000 --warmup 100 > $R/gpurun_out/trace_pack.log 2>&1 || { tail -5 $R/gpurun_out/trace_pack.log; exit 6; }
cd $R && python3 scripts/prof_summary.py gpurun_out/trace_pack --steps 4400 > gpurun_out/r4g_trace_pack.md && cat gpurun_out/r4g_trace_pack.md
