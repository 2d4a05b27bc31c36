#!/bin/bash
# soak: 1M steps of the one-GPU program, health words checked every 100k steps
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/mb/soak.py > gpurun_out/soak.txt 2>gpurun_out/soak.err; rc=$?
cat gpurun_out/soak.txt; [ $rc -ne 0 ] && tail -20 gpurun_out/soak.err; exit $rc
