# round 6: R16 tier gate for single frames (A/B builds base / gate 0 / gate 8192)
# over the bench frame (4032x3008) and configs[2] (8192^2), q50 and q90
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 50 90; do
  KB_Q=$q bash tools/kab.sh r6l_4k_q$q build_var/base build_var/g0 build_var/g8k || exit 1
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6l_8k_q$q build_var/base build_var/g0 build_var/g8k || exit 1
done
echo done
