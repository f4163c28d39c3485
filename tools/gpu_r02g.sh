#!/bin/bash
# r02g: generic-geometry kernels (runtime board, per-tile-count instantiations, padded filters):
# NN parity incl. the reference's templates on all five games, runner parity, player on GPU
set -o pipefail
T=gpurun_out/r02g
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests/test_nn_gpu.py tests/test_runner_gpu.py tests/test_player_gpu.py -v -s --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
echo ALL OK
