#!/bin/bash
# Round 5: what does fc2's deferred segment (with the head epilogue) cost the carrying
# launch?  MB_HF with both segments, fc1's only, fc2's only.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for o in "" 0 1; do
  MB_HF=1 MB_HF_ONLY=$o timeout -k 10 200 python3 scripts/microbench.py --reps 300 > gpurun_out/r5hf_$o.txt 2>&1 || { tail -5 gpurun_out/r5hf_$o.txt; exit 3; }
  echo "only=[$o] $(grep -E "HF:" gpurun_out/r5hf_$o.txt)"
done
