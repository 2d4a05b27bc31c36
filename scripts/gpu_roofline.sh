#!/bin/bash
# Roofline evidence: isolated kernel timings + two PMC passes (each its own run).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/microbench.py --reps 200 > gpurun_out/micro.txt 2>&1 || { tail -20 gpurun_out/micro.txt; exit 6; }
rm -rf $R/gpurun_out/rfA $R/gpurun_out/rfB
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE -f csv -d "$R/gpurun_out/rfA" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/rfA.log" 2>&1 || { echo "pass A failed"; tail -5 $R/gpurun_out/rfA.log; exit 7; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -f csv -d "$R/gpurun_out/rfB" -o run -- python3 "$R/scripts/microbench.py" --reps 5 > "$R/gpurun_out/rfB.log" 2>&1 || { echo "pass B failed"; tail -5 $R/gpurun_out/rfB.log; exit 8; }
cd $R && python scripts/roofline.py gpurun_out/rfA gpurun_out/rfB gpurun_out/micro.txt > gpurun_out/roofline.md && cat gpurun_out/roofline.md
