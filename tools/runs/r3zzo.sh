# K2 window size (2 / 8 tiles against 4) and length keys off, at 3 x 24 with the tier
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh default build_var/win2 build_var/win8 build_var/nomsz > gpurun_out/r3zzo_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zzo_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zzo_ab.txt
cat gpurun_out/r3zzo_ab.txt
