#!/bin/bash
# r03w: the driver's bench command (final tree), then the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
TAG=${1:-r03w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
timeout -k 10 580 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_trace.log; exit 1; }
find $T/trace -name "*kernel_trace.csv" -delete
find $T/trace -name "*kernel_stats.csv" -exec head -3 {} \;
echo ALL OK
