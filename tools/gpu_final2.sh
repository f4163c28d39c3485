#!/bin/bash
# Headline bench + rocprofv3 kernel-trace --stats of the SAME command (default args); the per-launch
# trace csv is deleted afterwards (hundreds of thousands of rows), the stats summary is kept.
set -o pipefail
TAG=${1:-r01i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 480 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o bench -- \
    python3 $R/bench.py > $R/gpurun_out/$TAG/bench_trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
find $R/gpurun_out/$TAG/trace -name "*kernel_trace.csv" -delete
tail -1 $R/gpurun_out/$TAG/bench_trace.log
echo ALL OK
