#!/bin/bash
# A/B: VALU conv pair (+ BN table by the last workgroup) vs the MFMA pair family.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/ab.txt
for r in 1 2 3; do
  for v in "" "CSA_CP_MFMA=1" "CSA_PAIR_BN_TAB=0"; do
    ms=$(env $v timeout -k 10 120 python bench.py --steps 3000 --warmup 300 | python -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])') || exit 1
    echo "[$v] $ms" | tee -a gpurun_out/ab.txt
  done
done
