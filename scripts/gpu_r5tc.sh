#!/bin/bash
# Round 5: stamps of pair workgroups with the BN tables, and the step trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 0; do
  CSA_PAIR_BN_TAB=$v MB_HF=1 MB_CP_BLOCKS=1,350,699 timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5tc_mb$v.txt 2>&1 || { tail -5 gpurun_out/r5tc_mb$v.txt; exit 4; }
  echo "tab=$v"; grep -E "HF:|pair alone block|updates block" gpurun_out/r5tc_mb$v.txt
done
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5tc_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python3 scripts/step_timeline.py $(find gpurun_out/r5tc_tr -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 4
for r in 1 2; do
  for v in 0 1; do
    a=$(CSA_PAIR_BN_TAB=$v timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(CSA_PAIR_BN_TAB=$v timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "tab=$v 20/5 $a 2000/200 $b"
  done
done
