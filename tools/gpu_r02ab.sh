#!/bin/bash
# r02ab: hoisted head 1x1 weights + pipelined initial-conv weights: NN GPU tests, timings, stamps
set -o pipefail
T=gpurun_out/${1:-r02ab}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_nn_gpu.py tests/test_nn_v2_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
bash tools/gpu_timing.sh $1/timing > $T/timing_run.txt 2>&1 || { echo "timing failed"; tail -5 $T/timing_run.txt; exit 1; }
grep -E 'N= 1024|fixed' $T/timing_run.txt
bash tools/gpu_stamps.sh $1/stamps > $T/stamps_run.txt 2>&1 || { echo "stamps failed"; exit 1; }
grep -E 'stamps|fixed' $T/stamps_run.txt
echo ALL OK
