#!/bin/bash
# Round-5 final tree: the driver's command (python bench.py), then the same under rocprofv3
# --kernel-trace --stats, then the PMC passes of the headline kernel (tools/gpu_pmc_r04.sh).
set -o pipefail
TAG=${1:-r05b}; PART=${2:-bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
# heartbeat under gpurun_out (long tests -- the oracle replays -- print nothing for minutes)
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$PART" = bench ]; then
  timeout -k 10 1000 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -5 $T/bench.log; exit 1; }
  grep "^{" $T/bench.log | tail -1 | cut -c1-400
elif [ "$PART" = trace ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
      python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_trace.log; exit 1; }
  find $T/trace -name "*kernel_trace.csv" -delete
  find $T/trace -name "*kernel_stats.csv" -exec head -5 {} \;
  grep "^{" $T/bench_trace.log | tail -1 | cut -c1-300
else
  bash $R/tools/gpu_pmc_r04.sh $TAG/pmc
fi
