#!/bin/bash
# NN-forward GPU pass: parity tests of every geometry + per-config kernel timing.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nn_gpu.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/nn_tests.log 2>&1 || { echo "nn tests failed"; tail -40 gpurun_out/nn_tests.log; exit 1; }
timeout -k 10 300 python tools/kernel_variants.py --configs ${KV_CONFIGS:-3,4,5} --batches ${KV_BATCHES:-64,256,1024} --variants default > gpurun_out/kv_cfg345.log 2>&1 || { echo kv failed; cat gpurun_out/kv_cfg345.log; exit 1; }
cat gpurun_out/kv_cfg345.log
echo ALL OK
