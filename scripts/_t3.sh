cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && mkdir -p gpurun_out/t3 && rm -f gpurun_out/t3/ab.log && \
DBG_IMPL=1 timeout -k 10 120 python scripts/_dbg_score.py > gpurun_out/t3/dbg.log 2>&1; grep -c "mismatches 0" gpurun_out/t3/dbg.log; \
for i in 1 0; do AB_IMPL=$i timeout -k 10 120 python scripts/ab_score.py >> gpurun_out/t3/ab.log 2>&1 || exit $?; AB_LD=100032 AB_IMPL=$i timeout -k 10 120 python scripts/ab_score.py >> gpurun_out/t3/ab.log 2>&1 || exit $?; done; grep -v "amdgpu.ids\|torch fill" gpurun_out/t3/ab.log
