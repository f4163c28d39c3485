#!/bin/bash
# r03y: the bench configuration's throughput curve on the final engine, 10-s intervals, 1000 s (one run)
set -o pipefail
T=gpurun_out/${1:-r03y}
mkdir -p $T
timeout -k 10 1090 python -u tools/steady_curve.py --seconds 1000 --interval 10 --out $T/curve.json > $T/curve.log 2>&1 || { echo "curve failed"; tail -5 $T/curve.log; exit 1; }
tail -3 $T/curve.log
echo ALL OK
