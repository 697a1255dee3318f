# round 6: code objects built for gfx950:xnack- (XNACK is off on these boxes)
# against the default gfx950 (xnack any): round-trip check + kernel times
# (chef-big q50) and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KB_Q=50 bash tools/kab.sh r6al_4k_q50 yuv-manipulations-2_amd build_var/xnackoff || exit 1
grep -hE "q50:|fdct_quant|huff_encode |huff_decode|compress wall" gpurun_out/kab_r6al_4k_q50.txt
bash tools/ab_bench.sh default build_var/xnackoff > gpurun_out/r6al_ab.txt 2>&1 || exit 1
cat gpurun_out/r6al_ab.txt
