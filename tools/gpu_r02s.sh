#!/bin/bash
# r02s: runner planes staged to HBM by DMA on a copy stream: runner / self-play / bench GPU tests,
# smoke, then the bench with and without the staging (GZ_RUNNER_ZERO_COPY=1), no CPU baseline
set -o pipefail
T=gpurun_out/${1:-r02s}
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests/test_runner_gpu.py tests/test_selfplay_gpu.py tests/test_bench_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench_dma.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_dma.log; exit 1; }
tail -1 $T/bench_dma.log | cut -c1-200
GZ_RUNNER_ZERO_COPY=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench_zc.log 2>&1 || { echo "bench zc failed"; tail -20 $T/bench_zc.log; exit 1; }
tail -1 $T/bench_zc.log | cut -c1-200
echo ALL OK
