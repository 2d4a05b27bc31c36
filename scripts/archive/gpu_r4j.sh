#!/bin/bash
# A/B: s_setprio(3) on the pair-backward waves of the launch that carries the dense updates.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CSA_HF_PRIO=1 timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py -x -q -k "horizontal_fusion" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4j_t.log 2>&1 || { tail -30 gpurun_out/r4j_t.log; exit 3; }
echo tests ok
b() {
env $1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4j_b.json 2>> gpurun_out/r4j.err || { tail -20 gpurun_out/r4j.err; exit 4; }
echo "$1 $(python3 -c "import json;d=json.load(open('gpurun_out/r4j_b.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2 3; do b CSA_HF_PRIO=0; b CSA_HF_PRIO=1; done
