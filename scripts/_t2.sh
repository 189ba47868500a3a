cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp && mkdir -p gpurun_out/t2 && \
AB_SHAPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t2/prof1 -o run -- python3 scripts/ab_topk.py > gpurun_out/t2/prof1.log 2>&1 && \
AB_SHAPE=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t2/prof2 -o run -- python3 scripts/ab_topk.py > gpurun_out/t2/prof2.log 2>&1; echo rc=$?
