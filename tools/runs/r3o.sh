# round 3: the decoder's time split after the symbol-loop rewrite (MYYUV_K5_EXP
# ablations: 1 no symbol decode, 2 no table parse either, 3 no transform)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or decompress or golden or sparse or error or irregular or tiled or noise" > gpurun_out/r3o_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
timeout -k 10 600 python3 tools/k1_ab.py build_var/r3base default build_var/k5x1 build_var/k5x2 build_var/k5x3 > gpurun_out/r3o_kab.txt 2>&1; cat gpurun_out/r3o_kab.txt
