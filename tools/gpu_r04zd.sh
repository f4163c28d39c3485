#!/bin/bash
# r04zd: phase B of the two-phase dense heads from registers (register softmax, value outputs in one
# pass; tools/kexp lib_base) against the three-pass LDS softmax (lib_phasebold): cfg2 bit-identity,
# timing, stamps; then the NN / runner GPU tests on the product library
# (a record: the change was reverted after this run and the phasebold patch dropped with it)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04c.sh r04zd phasebold || exit 1
( while sleep 45; do date +%T >> gpurun_out/r04zd/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_v2_gpu.py tests/test_bench_shape_gpu.py tests/test_runner_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04zd/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r04zd/tests.log | head; tail -3 gpurun_out/r04zd/tests.log; exit 1; }
tail -1 gpurun_out/r04zd/tests.log
