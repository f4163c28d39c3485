#!/bin/bash
# r04z: the two-image kernels' epilogues inside the conv's last k-step (tools/kexp lib_base) against
# after the conv (lib_epioff): cfg2 bit-identity, timing, stamps; then the NN GPU tests on the
# product library (epilogues inside)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04c.sh r04z epioff || exit 1
( while sleep 45; do date +%T >> gpurun_out/r04z/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py tests/test_runner_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04z/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r04z/tests.log | head; tail -3 gpurun_out/r04z/tests.log; exit 1; }
tail -1 gpurun_out/r04z/tests.log
