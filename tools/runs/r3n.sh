# round 3: streamlined decoder symbol loop (unconditional state, failed lanes
# re-decoded bit-serially for the exact code); exit test every 8/4/2/1 positions
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or decompress or golden or sparse or error or irregular or tiled or noise" > gpurun_out/r3n_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
timeout -k 10 600 python3 tools/k1_ab.py build_var/r3base build_var/dg8 build_var/dg4 build_var/dg2 build_var/dg1 > gpurun_out/r3n_kab.txt 2>&1; cat gpurun_out/r3n_kab.txt
