#!/bin/bash
# r02aa: kernel phase stamps, runner / self-play GPU tests, bench (no CPU baseline)
set -o pipefail
T=gpurun_out/${1:-r02aa}
mkdir -p $T
bash tools/gpu_stamps.sh $1/stamps > $T/stamps_run.txt 2>&1 || { echo "stamps failed"; tail -5 $T/stamps_run.txt; exit 1; }
grep -E 'stamps|fixed' $T/stamps_run.txt
timeout -k 10 400 python -u -m pytest tests/test_runner_gpu.py tests/test_selfplay_gpu.py -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $T/tests.log | head -20; exit 1; }
tail -1 $T/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-160
echo ALL OK
