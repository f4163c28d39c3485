#!/bin/bash
# GPU pass after a kernel/runner change: all GPU tests + smoke, forward timing by launch size,
# a short and a default bench.
set -o pipefail
T=${1:-r01m}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head; tail -5 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 200 python __graft_entry__.py > gpurun_out/$T/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 200 python tools/kernel_variants.py --configs 2,3 --batches 256,300,384,512,640,768,1024 --variants default > gpurun_out/$T/kv.log 2>&1 || { echo kv failed; exit 1; }
cat gpurun_out/$T/kv.log
timeout -k 10 480 python bench.py > gpurun_out/$T/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log
echo ALL OK
