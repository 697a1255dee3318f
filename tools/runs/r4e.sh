# round 4: K2 variants — the DC of single-class runs from LDS (k2dc), and an
# LDS cache of the non-single blocks' nonzero rows kept at classification
# (8 / 16 / 20 KB per workgroup, with the DC) — and K4 with 2 / 4 tiles per
# workgroup: bench A/B (3 alternating rounds; the untimed pass checks every
# stream against the pinned bytes) and per-kernel times at 24-frame launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 bash tools/ab_bench.sh default build_var/k2dc build_var/k2c8 build_var/k2c16 build_var/k2c20 build_var/k4t2 build_var/k4t4 > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4e_ab.txt && cat gpurun_out/r4e_ab.txt
K1AB_B=24 timeout -k 10 400 python3 tools/k1_ab.py default build_var/k2dc build_var/k2c16 build_var/k2c20 build_var/k4t2 build_var/k4t4 > gpurun_out/r4e_kab.txt 2>&1; cat gpurun_out/r4e_kab.txt
