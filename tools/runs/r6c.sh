# round 6: trace the host-batch pipeline on the big frame (r6b hung there)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_PIPE_TRACE=1 timeout -k 10 100 python -u -m pytest tests/test_gpu_host_batch.py -k "big and split" -x -s -v --timeout 90 --timeout-method thread > gpurun_out/r6c.log 2>&1
echo rc=$?
tail -40 gpurun_out/r6c.log
