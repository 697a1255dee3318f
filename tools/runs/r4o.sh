# round 4: K1's quad exchanges as DPP quad_perm moves instead of ds_bpermute
# and the msz product as v_pk_mul_lo_u16 (k1both), against the in-tree build;
# per-kernel times and the bench; then tools/runs/r4p.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1AB_B=24 timeout -k 10 300 python3 tools/k1_ab.py default build_var/k1both > gpurun_out/r4o_kab.txt 2>&1; cat gpurun_out/r4o_kab.txt
timeout -k 10 400 bash tools/ab_bench.sh default build_var/k1both > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4o_ab.txt && cat gpurun_out/r4o_ab.txt
bash tools/runs/r4p.sh
