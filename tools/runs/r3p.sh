# round 3: split decoder (K5 -> K6) times with the new symbol loop, K5 at 5 / 6 waves per SIMD
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MYYUV_DECODER=split timeout -k 10 600 python3 tools/k1_ab.py default build_var/k5s6 build_var/r3base > gpurun_out/r3p_kab.txt 2>&1; cat gpurun_out/r3p_kab.txt
