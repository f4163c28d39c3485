#!/bin/bash
# Aged benches of BASELINE configs (cfg 3-5) under rocprofv3 --kernel-trace --stats: the bench's JSON
# line (games/sec after aging) and the per-kernel summary of the same run.
# usage: bash tools/gpu_cfg_aged.sh TAG "3 4" [age_seconds]
set -o pipefail
TAG=${1:-r03o}
CFGS=${2:-"3"}
AGE=${3:-240}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d $T/cfg$c -o cfg$c -- \
      python3 $R/bench.py --gpus 1 --config $c --steps 10 --warmup 3 --age-seconds $AGE --no-cpu-baseline \
      > $T/bench_cfg$c.log 2>&1 || { echo "cfg$c failed"; tail -5 $T/bench_cfg$c.log; exit 1; }
  find $T/cfg$c -name "*kernel_trace.csv" -delete
  grep "^{" $T/bench_cfg$c.log | tail -1 | cut -c1-300
  find $T/cfg$c -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-200
done
echo ALL OK
