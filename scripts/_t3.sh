cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && mkdir -p gpurun_out/t3 && rm -f gpurun_out/t3/ab.log && \
timeout -k 10 120 python scripts/_dbg_score.py > gpurun_out/t3/dbg.log 2>&1; grep -c "mismatches 0" gpurun_out/t3/dbg.log; \
timeout -k 10 200 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_score_topk_gpu.py -k variants > gpurun_out/t3/test.log 2>&1; tail -1 gpurun_out/t3/test.log; \
for f in 1 0; do for a in 0 1 4; do AB_FLAGS=$f AB_ABLATE=$a timeout -k 10 120 python scripts/ab_score.py >> gpurun_out/t3/ab.log 2>&1 || exit $?; done; done; grep -v "amdgpu.ids\|torch fill" gpurun_out/t3/ab.log
