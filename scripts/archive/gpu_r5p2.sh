#!/bin/bash
# Round 5: packed K = 4 / 8 at the 32-step graphs, with and without horizontal fusion (+ the
# tail program) in the packed profile; then the DP ":hf" kernel trace (profiles/r5_dp_trace.md).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for h in 0 1; do for j in 4 8; do
  CSA_PACKED_HFUSE=$h timeout -k 10 150 python3 bench.py --jobs $j --steps 2048 --warmup 256 > gpurun_out/r5p2_h${h}_j$j.json 2>> gpurun_out/r5p2.err || exit 3
  echo "hfuse=$h jobs=$j $(grep -o '"value": [0-9.]*' gpurun_out/r5p2_h${h}_j$j.json)"
done; done
bash scripts/gpu_r5t2.sh
