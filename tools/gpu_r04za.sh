#!/bin/bash
# r04za: the split two-image epilogues' swapped 16-byte stores (tools/kexp lib_base, kStoreSwap) against
# the two 8-byte stores per lane (lib_swapoff): cfg2 bit-identity, timing, stamps; then the NN / runner
# GPU tests on the product library (swapped stores)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04c.sh r04za swapoff || exit 1
( while sleep 45; do date +%T >> gpurun_out/r04za/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_v2_gpu.py tests/test_bench_shape_gpu.py tests/test_runner_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04za/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r04za/tests.log | head; tail -3 gpurun_out/r04za/tests.log; exit 1; }
tail -1 gpurun_out/r04za/tests.log
