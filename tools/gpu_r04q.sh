#!/bin/bash
# r04q: an 18-minute steady-state curve of the bench's workload (tools/steady_curve.py), per-interval
# rates and per-ordinal game costs (the stationary estimates of DESIGN.md section 6 over time)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04q
mkdir -p $T
cd $R
timeout -k 10 1150 python -u tools/steady_curve.py --seconds 1080 --interval 40 --out $T/curve.json > $T/curve.log 2>&1 || { echo "curve failed"; tail -5 $T/curve.log; exit 1; }
tail -2 $T/curve.log | cut -c1-300
echo ALL OK
