#!/bin/bash
# Round 5: kernel traces of the step with and without the pair-backward tail.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for t in 0 1; do
  cd /tmp && CSA_PAIR_TAIL=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5h_prof$t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 500 --warmup 50 > $GRAFT_REPO_ROOT/gpurun_out/r5h_b$t.json 2>/dev/null || exit 6
  cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/r5h_prof$t -name "*kernel_stats.csv" | head -1); echo "== tail=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5h_b$t.json)"; head -12 "$f" | cut -d, -f1-4 | cut -c1-150
done
