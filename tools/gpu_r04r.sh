#!/bin/bash
# r04r: the two-pass kernel's direct lo stores (lib_full_base) vs the image + sweep scheme
# (lib_full_lodirectoff): cfg4 / cfg5 bit-identity + timing, then the cfg4 NN / runner tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04d.sh r04r full_lodirectoff || exit 1
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_runner_deep_gpu.py tests/test_bench_shape_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04r/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r04r/tests.log | head; tail -3 gpurun_out/r04r/tests.log; exit 1; }
tail -1 gpurun_out/r04r/tests.log
