#!/bin/bash
# r03k: fast-path verification test (register spin runs replayed), smoke, the driver's bench command,
# and the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
TAG=${1:-r03k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_runner_verify_gpu.py -v -s --timeout 380 --timeout-method thread > $T/verify_test.log 2>&1 || { echo "verify test failed"; grep -E "FAILED|Error|assert|mismatch" $T/verify_test.log | head; exit 1; }
grep -E "passed|failed" $T/verify_test.log | tail -1
timeout -k 10 200 python -u __graft_entry__.py > $T/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $T/smoke.log; exit 1; }
grep smoke: $T/smoke.log
timeout -k 10 420 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d $T/trace -o bench -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $T/bench_trace.log; exit 1; }
find $T/trace -name "*kernel_trace.csv" -delete
find $T/trace -name "*kernel_stats.csv" -exec head -4 {} \;
echo ALL OK
