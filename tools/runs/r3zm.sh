# wave issue priorities (s_setprio) for the latency-bound kernels in the 4 x 8 pipeline:
# pw3 = overflow passes 3; pall = + scans 3, stream_out 2; pdec = + decoder 1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh default build_var/pw3 build_var/pall build_var/pdec > gpurun_out/r3zm_ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r3zm_ab.txt; exit 1; }
cp gpurun_out/ab_bench.txt gpurun_out/r3zm_ab.txt
cat gpurun_out/r3zm_ab.txt
