#!/bin/bash
# GPU validation pass used during development: gpu tests, smoke, short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -s > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 150 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 420 python bench.py "$@" > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; exit 1; }
echo ALL OK
