#!/bin/bash
# Round 5: the tail's finish ticket relaxed (no L2 write-back on the critical path) and no
# acquire in the staging tails.  Numerics, carrier trace mean, same-box A/B vs ab_old.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py tests/test_deterministic.py tests/test_gpu_dp_overlap.py tests/test_gpu_platform.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5rl_t.txt 2>&1 || { tail -30 gpurun_out/r5rl_t.txt; exit 3; }
tail -1 gpurun_out/r5rl_t.txt
MB_HF=1 MB_TAIL=1 MB_EDGES=828,1808 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5rl_mb.txt 2>&1 || { tail -5 gpurun_out/r5rl_mb.txt; exit 4; }
grep -E "life|blocks \[" gpurun_out/r5rl_mb.txt
rm -rf gpurun_out/r5rl_tr
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5rl_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1) || exit 6
grep -h conv_pair_bwd_upd $(find gpurun_out/r5rl_tr -name "*kernel_stats.csv") | cut -d, -f1-6
for r in 1 2 3; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    a=$(cd $d && timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(cd $d && timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "$v 20/5 $a 2000/200 $b"
  done
done
