#!/bin/bash
# PMC counters per kernel (--pmc only with --kernel-trace; never with sys/runtime traces).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=${1:-pmc2}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --backend hip --steps 30 --warmup 5 --no-graph > "$GRAFT_REPO_ROOT/gpurun_out/$OUT.log" 2>&1
echo rc=$?
