#!/bin/bash
# configs 3-5 through the same runner path (short windows from the opening, no aging, no CPU baseline)
set -o pipefail
T=gpurun_out/${1:-cfgs2}
mkdir -p $T
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --age-seconds 0 --steps 6 --warmup 2 > $T/cfg$c.log 2>&1 || { echo "cfg$c failed"; tail -5 $T/cfg$c.log; exit 1; }
  tail -1 $T/cfg$c.log | cut -c1-200
done
echo ALL OK
