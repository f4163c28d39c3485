#!/bin/bash
# Launch-batching A/B: runner tests, then the same short bench window with and without holding
# launches for min_launch_rows.
set -o pipefail
mkdir -p gpurun_out/lb
timeout -k 10 300 python -u -m pytest tests/test_selfplay_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/lb/tests.log 2>&1 || { echo "selfplay tests failed"; tail -30 gpurun_out/lb/tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 3000 --no-cpu-baseline --min-launch-rows 0 > gpurun_out/lb/a.log 2>&1 || { echo "A failed"; tail gpurun_out/lb/a.log; exit 1; }
tail -1 gpurun_out/lb/a.log
timeout -k 10 300 python bench.py --steps 3000 --no-cpu-baseline > gpurun_out/lb/b.log 2>&1 || { echo "B failed"; tail gpurun_out/lb/b.log; exit 1; }
tail -1 gpurun_out/lb/b.log
timeout -k 10 300 python bench.py --steps 3000 --no-cpu-baseline --min-launch-rows 1024 --max-launch-wait-us 3000 > gpurun_out/lb/c.log 2>&1 || { echo "C failed"; tail gpurun_out/lb/c.log; exit 1; }
tail -1 gpurun_out/lb/c.log
echo ALL OK
