#!/bin/bash
# bench A/B on one box (no CPU baseline): 2 vs 3 pools per engine thread, twice each, interleaved
set -o pipefail
T=gpurun_out/${1:-knobs3}
mkdir -p $T
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/p2_$i.log 2>&1 || { echo "p2 failed"; exit 1; }
  tail -1 $T/p2_$i.log | cut -c1-160
  timeout -k 10 450 python -u bench.py --no-cpu-baseline --pools 3 > $T/p3_$i.log 2>&1 || { echo "p3 failed"; exit 1; }
  tail -1 $T/p3_$i.log | cut -c1-160
done
echo ALL OK
