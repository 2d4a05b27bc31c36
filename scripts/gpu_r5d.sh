#!/bin/bash
# Round 5: co-scheduling probe of processes sharing one GPU (scripts/coschedule_probe.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r5d.jsonl; : > $out
timeout -k 10 120 python3 scripts/coschedule_probe.py --world 2 --delay 1.0 >> $out 2>> gpurun_out/r5d.err || exit 3
timeout -k 10 120 python3 scripts/coschedule_probe.py --world 2 --delay 1.0 --busy 300 >> $out 2>> gpurun_out/r5d.err || exit 4
timeout -k 10 120 python3 scripts/coschedule_probe.py --world 4 --delay 1.0 >> $out 2>> gpurun_out/r5d.err || exit 5
cat $out | cut -c1-1500
