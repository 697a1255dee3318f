# round 6: integer instruction-form issue costs (tools/ubench/iforms.hip), and
# the decoder's symbol loop in full-rate forms (MYYUV_K5_FORMS) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench/iforms > gpurun_out/r6g_iforms.txt 2>&1; cat gpurun_out/r6g_iforms.txt
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/k5base > gpurun_out/r6g_kab.txt 2>&1; cat gpurun_out/r6g_kab.txt
timeout -k 10 500 bash tools/ab_bench.sh default build_var/k5base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r6g_ab.txt && cat gpurun_out/r6g_ab.txt
