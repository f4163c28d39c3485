#!/bin/bash
# r03d: exact-round launch composition (split pools): runner oracle tests, bench A/B split vs subset
set -o pipefail
T=gpurun_out/${1:-r03d}
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests/test_runner_gpu.py -x -v --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench_split.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_split.log; exit 1; }
tail -1 $T/bench_split.log | cut -c1-300
GZ_RUNNER_COMPOSE=subset timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_subset.log 2>&1 || { echo "bench subset failed"; tail -20 $T/bench_subset.log; exit 1; }
tail -1 $T/bench_subset.log | cut -c1-300
echo ALL OK
