# round 4: K1 lists its unproven units 64 at a time per wave (one atomic per
# wave and flush; at q90 one counter took 47k atomics per 8192x8192 frame),
# DPP quad exchanges and the packed msz product on by default: every GPU test,
# smoke, configs[2] (q50, q90: trace and traffic), and the bench against the
# same build with per-unit atomics (build_var/prevlist)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r4q_tests.log; exit 1; }
tail -1 gpurun_out/r4q_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4q_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/r4q_smoke.log; exit 1; }
echo smoke ok
bash tools/cfg2_profile.sh r4qcfg2 10 > gpurun_out/r4q_cfg2.txt 2>&1 && echo CFG2_OK
timeout -k 10 500 bash tools/ab_bench.sh default build_var/prevlist > /dev/null && cp gpurun_out/ab_bench.txt gpurun_out/r4q_ab.txt && cat gpurun_out/r4q_ab.txt
