# round 5 (final build): each kernel's marginal cost in the bench's pipeline
# (4 x 24 launch groups; tools/kskip.py skips one kernel's launches at a time)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KSKIP_NF=4 timeout -k 10 600 python3 tools/kskip.py > gpurun_out/r5bg_kskip.txt 2>&1; cat gpurun_out/r5bg_kskip.txt
