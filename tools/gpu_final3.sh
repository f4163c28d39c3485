#!/bin/bash
# Round-end pass: GPU tests + smoke, headline bench, rocprofv3 kernel-trace --stats of the same command.
set -o pipefail
TAG=${1:-r01o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/$TAG/tests.log | head; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 200 python __graft_entry__.py > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 480 python bench.py > gpurun_out/$TAG/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/trace -o bench -- \
    python3 $R/bench.py > $R/gpurun_out/$TAG/bench_trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
find $R/gpurun_out/$TAG/trace -name "*kernel_trace.csv" -delete
echo ALL OK
