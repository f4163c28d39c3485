#!/bin/bash
# r04h: PMC passes of the asm-chain split trunk (1024 rows), then the driver's bench command
set -o pipefail
TAG=${1:-r04h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
bash tools/gpu_pmc_r04.sh $TAG/pmc > $T/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $T/pmc.log; exit 1; }
grep -A14 "trunk_kernel" $T/pmc/summary.txt
cd $R
timeout -k 10 900 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-600
echo ALL OK
