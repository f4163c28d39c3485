#!/bin/bash
# GPU pass for the non-headline configs: self-play GPU tests, then short self-play benches of
# BASELINE configs 3-5 through the same runner (memory-bounded: few games, few steps for cfg4/5,
# whose trees hold up to ~2,000 children per node).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_selfplay_gpu.py -k other_games -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/selfplay_tests.log 2>&1 || { echo "selfplay tests failed"; tail -30 gpurun_out/selfplay_tests.log; exit 1; }
timeout -k 10 300 python bench.py --config 3 --steps 300 --warmup 20 --pools 2 --cpu-baseline-seconds 15 \
    > gpurun_out/bench_cfg3.log 2>&1 || { echo "cfg3 bench failed"; tail -20 gpurun_out/bench_cfg3.log; exit 1; }
timeout -k 10 300 python bench.py --config 4 --steps 60 --warmup 5 --threads 8 --pools 1 --cpu-baseline-seconds 15 \
    > gpurun_out/bench_cfg4.log 2>&1 || { echo "cfg4 bench failed"; tail -20 gpurun_out/bench_cfg4.log; exit 1; }
timeout -k 10 300 python bench.py --config 5 --steps 60 --warmup 5 --threads 8 --pools 1 --cpu-baseline-seconds 15 \
    > gpurun_out/bench_cfg5.log 2>&1 || { echo "cfg5 bench failed"; tail -20 gpurun_out/bench_cfg5.log; exit 1; }
for c in 3 4 5; do tail -1 gpurun_out/bench_cfg$c.log; done
echo ALL OK
