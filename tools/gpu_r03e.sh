#!/bin/bash
# r03e: new parity tests (bench shape, deep configs on bench weights, generation roll, runner
# fast-path verification), runner oracle tests, bench A/B exact-round split vs subset composition
set -o pipefail
T=gpurun_out/${1:-r03e}
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests/test_bench_shape_gpu.py tests/test_runner_roll_gpu.py tests/test_runner_gpu.py -v -s --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $T/tests.log | head -20; exit 1; }
grep -E "passed|failed" $T/tests.log | tail -1
timeout -k 10 500 python -u -m pytest tests/test_runner_verify_gpu.py -x -v -s --timeout 450 --timeout-method thread > $T/verify.log 2>&1 || { echo "verify failed"; tail -30 $T/verify.log; exit 1; }
grep -E "passed|failed" $T/verify.log | tail -1
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench_split.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_split.log; exit 1; }
tail -1 $T/bench_split.log | cut -c1-300
GZ_RUNNER_COMPOSE=subset timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_subset.log 2>&1 || { echo "bench subset failed"; tail -20 $T/bench_subset.log; exit 1; }
tail -1 $T/bench_subset.log | cut -c1-300
echo ALL OK
