#!/bin/bash
# r02w: round-filling launch trim: runner GPU tests, then the bench with the new trim and with the
# legacy whole-wave trim (GZ_RUNNER_LEGACY_TRIM=1), no CPU baseline
set -o pipefail
T=gpurun_out/${1:-r02w}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_runner_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench_fill.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_fill.log; exit 1; }
tail -1 $T/bench_fill.log | cut -c1-160
GZ_RUNNER_LEGACY_TRIM=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench_legacy.log 2>&1 || { echo "bench legacy failed"; tail -20 $T/bench_legacy.log; exit 1; }
tail -1 $T/bench_legacy.log | cut -c1-160
echo ALL OK
