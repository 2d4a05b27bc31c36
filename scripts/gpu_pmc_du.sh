#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt" 2>&1
echo "list rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_du1" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/microbench.py" --reps 20 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_du1.log" 2>&1
echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_du2" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/microbench.py" --reps 20 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_du2.log" 2>&1
echo "pmc2 rc=$?"
