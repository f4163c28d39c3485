#!/bin/bash
# r03zc: the bench configuration's curve with the unique-states filters cleared every 120 s (the
# reference worker clears them at every new generation, worker.py:160), 600 s (one run)
set -o pipefail
T=gpurun_out/${1:-r03zc}
mkdir -p $T
timeout -k 10 690 python -u tools/steady_curve.py --seconds 600 --interval 10 --roll-seconds 120 --out $T/curve.json > $T/curve.log 2>&1 || { echo "curve failed"; tail -5 $T/curve.log; exit 1; }
tail -3 $T/curve.log
echo ALL OK
