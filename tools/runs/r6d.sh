# round 6: which host-batch calls differ on the big frame (diagnostic)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag/host_batch_check.py > gpurun_out/r6d.log 2>&1
echo rc=$?
cat gpurun_out/r6d.log
