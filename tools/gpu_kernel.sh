#!/bin/bash
# Kernel iteration pass: NN parity tests, then forward timing of cfg2 (and cfg1/3) variants.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/nn_tests.log 2>&1 || { echo "nn tests failed"; tail -40 gpurun_out/nn_tests.log; exit 1; }
timeout -k 10 200 python tools/kernel_variants.py --configs ${KV_CONFIGS:-1,2,3} --batches ${KV_BATCHES:-256,512,1024} \
    --variants ${KV_VARIANTS:-default,11,21} > gpurun_out/kv.log 2>&1 || { echo kv failed; cat gpurun_out/kv.log; exit 1; }
cat gpurun_out/kv.log
timeout -k 10 200 python tools/kernel_breakdown.py --variants 11,21 --batches 256,512 > gpurun_out/breakdown.log 2>&1 || { echo bd failed; exit 1; }
cat gpurun_out/breakdown.log
echo ALL OK
