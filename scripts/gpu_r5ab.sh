#!/bin/bash
# Round 5: same-box A/B of the whole step, the revision at the start of this session's
# kernel work (ab_old/, built from 4c08035, not tracked) against the working tree.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for v in old new; do
    d=.; [ $v = old ] && d=ab_old
    a=$(cd $d && timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    b=$(cd $d && timeout -k 10 120 python3 bench.py --steps 2000 --warmup 200 | grep -o '"ms_per_step": [0-9.]*') || exit 5
    echo "$v 20/5 $a 2000/200 $b"
  done
done
