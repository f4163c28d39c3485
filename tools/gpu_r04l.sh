#!/bin/bash
# r04l: output staging for large policies (runner.hip) + the initial conv's hoisted weights / single
# im2col zeroing: the deep runner tests (amazons = output staging, replayed through the oracle), the
# NN parity tests, cfg2 timing + stamps against r04k's base (tools/kexp/lib_base), cfg5 aged bench
# under rocprofv3 --stats (heads share of GPU time)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04l
mkdir -p $T
cd $R
timeout -k 10 600 python -u -m pytest tests/test_runner_deep_gpu.py tests/test_nn_gpu.py tests/test_bench_shape_gpu.py -x -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
bash tools/gpu_r04c.sh r04l conv0 > $T/kexp.log 2>&1 || { echo "kexp failed"; tail -5 $T/kexp.log; exit 1; }
cat $T/kexp.log
bash tools/gpu_cfg_aged.sh r04l "5" 60
