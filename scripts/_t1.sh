cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && mkdir -p gpurun_out/t1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_score_topk_gpu.py tests/test_sasrec_gpu.py tests/test_evaluate_gpu.py > gpurun_out/t1/topk.log 2>&1; rc=$?; tail -5 gpurun_out/t1/topk.log; \
if [ $rc -eq 0 ]; then timeout -k 10 300 python bench.py --skip sasrec,c4 --no-cpu-baseline --steps 5 > gpurun_out/t1/bench.log 2>&1; echo bench rc=$?; tail -c 1200 gpurun_out/t1/bench.log; fi
