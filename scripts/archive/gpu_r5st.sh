#!/bin/bash
# Round 5 (final): one-GPU step trace (rocprofv3 kernel trace, two steps) for
# profiles/r5_step_trace.md.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5st -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1100 --warmup 100 > /dev/null 2>&1 || exit 6
cd $GRAFT_REPO_ROOT && python3 scripts/step_timeline.py $(find gpurun_out/r5st -name "*kernel_trace.csv" | head -1) --skip 1000 --steps 3
python3 scripts/prof_summary.py $(find gpurun_out/r5st -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -12 || true
