#!/bin/bash
# r02b: steady-state curve (spin fast path engine), then reversi runner-vs-oracle + drop-in GPU tests
set -o pipefail
T=gpurun_out/r02b
mkdir -p $T
timeout -k 10 470 python -u tools/steady_curve.py --seconds 400 --interval 10 --pools 2 --out $T/curve_p2.json > $T/curve_p2.log 2>&1 || { echo "curve failed"; tail -20 $T/curve_p2.log; exit 1; }
tail -3 $T/curve_p2.log
timeout -k 10 900 python -u -m pytest tests/test_runner_gpu.py "tests/test_selfplay_gpu.py::test_dropin_supervisor_gpu_matches_oracle" -k "reversi or dropin" -x -v -s --timeout 850 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; tail -40 $T/tests.log; exit 1; }
grep -E "passed|failed|identical" $T/tests.log | tail -8
echo ALL OK
