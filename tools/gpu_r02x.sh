#!/bin/bash
# r02x: subset-sum launch composition: runner GPU tests, then the bench (no CPU baseline)
set -o pipefail
T=gpurun_out/${1:-r02x}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_runner_gpu.py tests/test_selfplay_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench_subset.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_subset.log; exit 1; }
tail -1 $T/bench_subset.log | cut -c1-160
echo ALL OK
