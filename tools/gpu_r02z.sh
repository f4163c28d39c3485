#!/bin/bash
# r02z: launch-size knob with the round-filling composition: min_launch_rows 1536 and 1280 (no CPU baseline)
set -o pipefail
T=gpurun_out/${1:-r02z}
mkdir -p $T
timeout -k 10 400 python -u bench.py --no-cpu-baseline --min-launch-rows 1536 > $T/rows1536.log 2>&1 || { echo "1536 failed"; exit 1; }
tail -1 $T/rows1536.log | cut -c1-160
timeout -k 10 400 python -u bench.py --no-cpu-baseline --min-launch-rows 1280 > $T/rows1280.log 2>&1 || { echo "1280 failed"; exit 1; }
tail -1 $T/rows1280.log | cut -c1-160
echo ALL OK
