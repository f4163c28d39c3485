#!/bin/bash
# r06z: the driver's command (python bench.py) on the final tree, then the same workload under
# rocprofv3 --kernel-trace --stats (the summary whose trunk average must agree with the bench's
# HIP events)
set -o pipefail
TAG=${1:-r06z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -5 $T/bench.log; exit 1; }
grep "^{" $T/bench.log | tail -1 | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_under_rocprof.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_under_rocprof.log; exit 1; }
find $T/trace -name "*kernel_trace.csv" -delete
find $T/trace -name "*kernel_stats.csv" -exec head -5 {} \;
grep "^{" $T/bench_under_rocprof.log | tail -1 | cut -c1-300
