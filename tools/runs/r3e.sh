# round 3: K1 cost of the nonzero map (pk_min vs SWAR row flags, map store to the sink) and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/k1_ab.py default build_var/swar build_var/nzmsink build_var/r2 > gpurun_out/r3e_k1ab.txt 2>&1 || { echo K1AB_FAILED; tail -5 gpurun_out/r3e_k1ab.txt; exit 1; }
cat gpurun_out/r3e_k1ab.txt
timeout -k 10 900 bash tools/ab_bench.sh default build_var/swar build_var/r2 && cp gpurun_out/ab_bench.txt gpurun_out/r3e_ab.txt
