# round 4: the fused decoder's fast inverse again, with its sums advanced
# together (fence16, as the exact path), built from e9eac8c's decoder:
# dec_fnl (no fix list: the ceiling), dec_f5 (5 waves, spills), dec_f4 (4
# waves); per-kernel times against the in-tree build; then each kernel's
# marginal cost in the bench shape (tools/kskip.py, 4 x 24)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/dec_fnl build_var/dec_f5 build_var/dec_f4 > gpurun_out/r4p_kab.txt 2>&1; cat gpurun_out/r4p_kab.txt
KSKIP_NF=4 timeout -k 10 500 python3 tools/kskip.py > gpurun_out/r4p_kskip.txt 2>&1; cat gpurun_out/r4p_kskip.txt
# k_fdct_fix with one-wave workgroups (fix1: smaller slots to find among the other launch groups' waves)
timeout -k 10 500 bash tools/ab_bench.sh default build_var/fix1 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4p_fix1_ab.txt && cat gpurun_out/r4p_fix1_ab.txt
