#!/bin/bash
# bench knob A/B on one box (no CPU baseline): default, 1536-row launches, 3 pools per thread
set -o pipefail
T=gpurun_out/${1:-knobs2}
mkdir -p $T
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/default.log 2>&1 || { echo "default failed"; exit 1; }
tail -1 $T/default.log | cut -c1-200
timeout -k 10 400 python -u bench.py --no-cpu-baseline --min-launch-rows 1536 > $T/rows1536.log 2>&1 || { echo "rows1536 failed"; exit 1; }
tail -1 $T/rows1536.log | cut -c1-200
timeout -k 10 400 python -u bench.py --no-cpu-baseline --pools 3 > $T/pools3.log 2>&1 || { echo "pools3 failed"; exit 1; }
tail -1 $T/pools3.log | cut -c1-200
echo ALL OK
