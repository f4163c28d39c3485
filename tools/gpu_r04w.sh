#!/bin/bash
# r04w (final tree): the driver's bench command under rocprofv3 --kernel-trace --stats
set -o pipefail
TAG=${1:-r04w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_trace.log; exit 1; }
find $T/trace -name "*kernel_trace.csv" -delete
find $T/trace -name "*kernel_stats.csv" -exec head -5 {} \;
grep "^{" $T/bench_trace.log | tail -1 | cut -c1-300
echo ALL OK
