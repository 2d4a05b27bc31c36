#!/bin/bash
# Round 5: kernel traces of BOTH ranks of a world-2 stall (each rank its own process under
# its own rocprofv3): which of the stalled rank's kernels is not running while the other
# rank's xGMI kernel spins — not dispatched (begins after the wait) or resident but starved?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export CSA_XGMI_TIMEOUT_S=3 LOCAL_WORLD_SIZE=2
port=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
for r in 0 1; do
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5t_prof$r -o run -- \
    python3 scripts/xgmi_stress.py --world 2 --steps 60 --chunk 1 --rank $r --port $port > gpurun_out/r5t_rank$r.log 2>&1 &
  pids[$r]=$!
done
wait ${pids[0]}; rc0=$?; wait ${pids[1]}; rc1=$?
echo "rc0=$rc0 rc1=$rc1"; grep -h '"rank"' gpurun_out/r5t_rank*.log | cut -c1-300
exit 0
