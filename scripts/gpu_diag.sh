cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag_group.py > gpurun_out/diag1.txt 2>&1 && CSA_STAGE_BATCH=0 timeout -k 10 200 python scripts/diag_group.py >> gpurun_out/diag1.txt 2>&1; cat gpurun_out/diag1.txt | grep stage
