#!/bin/bash
# rocprofv3 kernel traces of the world-1 DP programs (allreduce:hf, ps:hf, async_ps)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
for s in allreduce:hf ps:hf async_ps; do
  t=${s/:/_}
  rm -rf $R/gpurun_out/trdp_$t; cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trdp_$t -o run -- python3 $R/scripts/bench_dp1.py --strategy $s --steps 1000 --warmup 100 > $R/gpurun_out/trdp_$t.log 2>&1 || { tail -5 $R/gpurun_out/trdp_$t.log; exit 3; }
  cd $R && python3 scripts/prof_summary.py gpurun_out/trdp_$t --steps 1100 --top 12 > gpurun_out/trdp_$t.md || exit 4
done
