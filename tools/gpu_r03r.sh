#!/bin/bash
# r03r: PMC passes on the split trunk at 1024 rows, then the driver's bench command (new aging default)
set -o pipefail
TAG=${1:-r03r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
bash tools/gpu_pmc_fp32.sh $TAG/pmc > $T/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $T/pmc.log; exit 1; }
grep -E "traffic|wave cycles|MFMA|BANK|grid" $T/pmc.log | head -20
cd $R
timeout -k 10 560 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-300
echo ALL OK
