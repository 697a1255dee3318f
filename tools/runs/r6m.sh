# round 6: k_huff_encode_r16 without spills (131 VGPRs, 3 waves/SIMD) for
# single frames: A/B builds base / gate 0 / gate 0 + no spills / no spills
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 50 90; do
  KB_Q=$q bash tools/kab.sh r6m_4k_q$q build_var/base build_var/g0 build_var/g0w2 || exit 1
  KB_Q=$q KB_SIZE=8192x8192 bash tools/kab.sh r6m_8k_q$q build_var/base build_var/g0 build_var/g0w2 build_var/w2 || exit 1
done
echo done
