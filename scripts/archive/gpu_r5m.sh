#!/bin/bash
# Round 5: packed jobs (K sample-config jobs as branches of one graph): the packed profile
# with / without horizontal fusion + the pair-backward tail.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 4 8; do for hf in 0 1; do
  CSA_PACKED_HFUSE=$hf timeout -k 10 300 python3 bench.py --jobs $k --pack graph --steps 1000 --warmup 100 > gpurun_out/r5m_${k}_$hf.json 2>> gpurun_out/r5m.err || exit 3
  echo "K=$k hfuse=$hf $(grep -o '"value": [0-9.]*' gpurun_out/r5m_${k}_$hf.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5m_${k}_$hf.json)"
done; done
