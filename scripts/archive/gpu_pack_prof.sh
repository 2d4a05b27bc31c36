#!/bin/bash
# Kernel traces of the single job and of K packed jobs (one graph, K branches).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for K in ${KS:-1 4}; do
  rm -rf $R/gpurun_out/prof_pack$K
  if [ $K -eq 1 ]; then args=""; else args="--jobs $K --pack graph"; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_pack$K" -o run -- python3 "$R/bench.py" $args --steps 200 --warmup 20 > "$R/gpurun_out/prof_pack$K.txt" 2>&1) || { tail -20 $R/gpurun_out/prof_pack$K.txt; exit 5; }
  python scripts/trace_overlap.py gpurun_out/prof_pack$K --filter csa:: > gpurun_out/overlap$K.md && cat gpurun_out/overlap$K.md
done
