#!/bin/bash
# Round pass on one MI355X: every GPU test, the smoke, the driver's bench command, and the same
# command under rocprofv3 --kernel-trace --stats (summaries kept under gpurun_out/$TAG).
# usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r02f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head; exit 1; }
tail -1 $T/tests.log
timeout -k 10 300 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_trace.log; exit 1; }
find $T/trace -name "*kernel_trace.csv" -delete
find $T/trace -name "*kernel_stats.csv" -exec head -5 {} \;
echo ALL OK
