#!/bin/bash
# Round 5: root cause of the round-4 xGMI flag loss.  The overlapped all-reduce step with
# W ranks on one GPU, 300 steps, four variants: round-4 kernels (plain epoch loads) /
# round-5 kernels (agent-scope epochs), each without and with the co-resident block cap.
# A timed-out wait is bounded (5 s) and recorded, never a hang; every step has its own limit.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp CSA_XGMI_TIMEOUT_S=5
out=gpurun_out/r5b.jsonl; : > $out
R4=$PWD/cloud_server_amd/_lib/variants/libcsa_kernels_r4xgmi.so
for w in 2 4; do
  for lib in r4 r5; do
    for cap in 0 auto; do
      c=$cap; [ $cap = auto ] && c=$((640 / w / 8 * 8))
      if [ $lib = r4 ]; then L=$R4; else L=; fi
      CSA_KERNEL_LIB=$L CSA_XGMI_BLOCKS=$c timeout -k 10 200 python3 scripts/xgmi_stress.py --world $w --steps 300 >> $out 2>> gpurun_out/r5b.err
      rc=$?; echo "w=$w lib=$lib cap=$c rc=$rc"
      [ $rc -gt 1 ] && { tail -5 gpurun_out/r5b.err; exit $rc; }
    done
  done
done
exit 0
