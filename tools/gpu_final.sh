#!/bin/bash
# Round measurement pass: default bench (headline line), literal-mode bench, and a rocprofv3
# kernel-trace --stats of a shorter bench run (per-kernel average durations for profiles/).
set -o pipefail
TAG=${1:-r01g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 480 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
timeout -k 10 420 python bench.py --mode literal --no-cpu-baseline > gpurun_out/$TAG/bench_literal.log 2>&1 || { echo "literal bench failed"; tail -20 gpurun_out/$TAG/bench_literal.log; exit 1; }
tail -1 gpurun_out/$TAG/bench_literal.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3000 > $R/gpurun_out/$TAG/bench_trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
tail -1 $R/gpurun_out/$TAG/bench_trace.log
echo ALL OK
