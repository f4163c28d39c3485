#!/bin/bash
# r02c: fp32-mode NN parity + bench paths (1 rank, 2 ranks over gloo) + the driver's bench command
set -o pipefail
T=gpurun_out/r02c
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_gpu.py -v -s --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $T/tests.log | head -20; tail -30 $T/tests.log; exit 1; }
grep -E "passed|failed" $T/tests.log | tail -3
timeout -k 10 580 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log
echo ALL OK
