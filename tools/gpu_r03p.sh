#!/bin/bash
# r03p: the bench configuration's throughput curve from the opening, 10-s intervals, 660 s (one run)
set -o pipefail
T=gpurun_out/${1:-r03p}
mkdir -p $T
timeout -k 10 780 python -u tools/steady_curve.py --seconds 660 --interval 10 --out $T/curve.json > $T/curve.log 2>&1 || { echo "curve failed"; tail -5 $T/curve.log; exit 1; }
tail -3 $T/curve.log
echo ALL OK
