set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_known_answers.py -m gpu -x -q -k sorted --timeout 300 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -2 gpurun_out/r03x_tests.log
timeout -k 10 120 python3 tools/dec_time.py > gpurun_out/r03x_dec.txt 2>&1
MYYUV_DECODER=sorted timeout -k 10 120 python3 tools/dec_time.py >> gpurun_out/r03x_dec.txt 2>&1
cat gpurun_out/r03x_dec.txt
timeout -k 10 900 bash tools/ab_bench.sh default MYYUV_DECODER=sorted
