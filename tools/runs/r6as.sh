# round 6: device-link code-generation options (tools/build_variant.sh
# LINKFLAGS): cg1 -amdgpu-use-amdgpu-trackers=1, cg2
# -amdgpu-disable-unclustered-high-rp-reschedule=1, cg3 -misched-cluster=0,
# cg4 -amdgpu-schedule-relaxed-occupancy=1, cg5
# -amdgpu-disable-clustered-low-occupancy-reschedule=1: bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab_bench.sh default build_var/cg1 build_var/cg2 build_var/cg3 build_var/cg4 build_var/cg5 > gpurun_out/r6as_ab.txt 2>&1 || { cat gpurun_out/r6as_ab.txt; exit 1; }
cat gpurun_out/r6as_ab.txt
