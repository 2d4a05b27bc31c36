#!/bin/bash
# A/B: update workgroups first in the pair backward; 128-column dense backward blocks.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CSA_HF_UPD_FIRST=1 timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py -x -q -k "horizontal_fusion" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4i_t.log 2>&1 || { tail -30 gpurun_out/r4i_t.log; exit 3; }
CSA_DU_CS4=1 timeout -k 10 300 python3 -u -m pytest tests/test_hip_step.py -x -q -k "horizontal_fusion" -p no:cacheprovider --timeout 120 --timeout-method thread >> gpurun_out/r4i_t.log 2>&1 || { tail -30 gpurun_out/r4i_t.log; exit 3; }
echo tests ok
b() {
env $1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/r4i_b.json 2>> gpurun_out/r4i.err || { tail -20 gpurun_out/r4i.err; exit 4; }
echo "$1 $(python3 -c "import json;d=json.load(open('gpurun_out/r4i_b.json'));print(d['ms_per_step'], d['value'])")"
}
for r in 1 2 3; do b CSA_X=0; b CSA_HF_UPD_FIRST=1; b CSA_DU_CS4=1; done
