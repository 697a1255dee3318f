# round 4: K1's block-info store (r4k: K2 -43 us but K1 +60 us per 24-frame
# launch): all four lanes storing the same word (bsame), the same with the
# sink spread over 64 per-wave slots (bsink), 7-wave budget (bocc7), against
# r4k's in-tree build (lane 0 stores, the others to the sink) and the previous
# commit (base); then the fused decoder's fast inverse (tools/runs/r4m.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/bsame build_var/bsink build_var/bocc7 build_var/base > gpurun_out/r4l_kab.txt 2>&1; cat gpurun_out/r4l_kab.txt
timeout -k 10 400 bash tools/ab_bench.sh build_var/bsame build_var/base > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4l_ab.txt && cat gpurun_out/r4l_ab.txt
bash tools/runs/r4m.sh
