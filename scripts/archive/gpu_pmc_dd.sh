#!/bin/bash
# PMC passes over the microbench (each pass its own run; SQ <= 8, TA <= 2, TCC <= 4).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pdd1 $R/gpurun_out/pdd2
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY -f csv -d "$R/gpurun_out/pdd1" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/pdd1.log" 2>&1 || { echo "pass 1 failed"; tail -5 $R/gpurun_out/pdd1.log; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA -f csv -d "$R/gpurun_out/pdd2" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/pdd2.log" 2>&1 || { echo "pass 2 failed"; tail -5 $R/gpurun_out/pdd2.log; exit 8; }
echo done
