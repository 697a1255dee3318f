# round 4: K1 register pressure.  Per-kernel times (24-frame launches) of the
# in-tree fast transform (92 VGPRs), the column-sequential stage 2 (build_var/seq),
# the fast path with no exact path (build_var/fastonly, 64 VGPRs: the ceiling
# of a lower-pressure fast path; its output may differ) and round-3 K1
# (build_var/k2dc); then the bench-level A/B of the same
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/seq build_var/fastonly build_var/k2dc > gpurun_out/r4g_kab.txt 2>&1; cat gpurun_out/r4g_kab.txt
timeout -k 10 800 bash tools/ab_bench.sh default build_var/fastonly build_var/seq > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4g_ab.txt && cat gpurun_out/r4g_ab.txt
