#!/bin/bash
# PMC counters per kernel (one pass per counter set; --pmc only with --kernel-trace/--stats).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --backend hip --steps 30 --warmup 5 --no-graph > "$GRAFT_REPO_ROOT/gpurun_out/pmc1.log" 2>&1
echo rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hip2" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --backend hip --steps 300 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_hip2.log" 2>&1
echo rc=$?
ls -R "$GRAFT_REPO_ROOT/gpurun_out/pmc1" | head
