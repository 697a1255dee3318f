#!/bin/bash
# GPU parity tests, then kernel timing of the default build and any gpurun_var/* variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
VARS=$(ls -d gpurun_var/*/ 2>/dev/null | sed 's#/$##')
bash tools/kab.sh quick yuv-manipulations-2_amd $VARS && cat gpurun_out/kab_quick.txt
