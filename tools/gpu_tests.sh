#!/bin/bash
# Full GPU test pass + smoke (what the driver runs at round end).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_tests_all.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_all.log | head -20; tail -5 gpurun_out/gpu_tests_all.log; exit 1; }
tail -3 gpurun_out/gpu_tests_all.log
timeout -k 10 200 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo ALL OK
