# round 3: transform code shape — no accumulator fence in the zero-skipping loops
# (nofence), plus stage-1 accumulators in tile order (default); base = HEAD (dg2x)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or decompress or golden or sparse or tiled or noise or numerics or parity" > gpurun_out/r3r_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
timeout -k 10 600 python3 tools/k1_ab.py build_var/dg2x build_var/nofence default > gpurun_out/r3r_kab.txt 2>&1; cat gpurun_out/r3r_kab.txt
MYYUV_DECODER=split timeout -k 10 600 python3 tools/k1_ab.py build_var/dg2x build_var/nofence default > gpurun_out/r3r_kab_split.txt 2>&1; cat gpurun_out/r3r_kab_split.txt
