cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp && mkdir -p gpurun_out/t2 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t2/fwd -o run -- python3 scripts/prof_sas.py --forward-only 1 --B 512 --d 128 --n 200 --items 1000 --iters 10 > gpurun_out/t2/fwd.log 2>&1; echo rc=$?; python3 scripts/kstats.py gpurun_out/t2/fwd
