#!/bin/bash
# r03n: the driver's bench command (template mode) and a literal-mode bench line
set -o pipefail
TAG=${1:-r03n}
T=gpurun_out/$TAG
mkdir -p $T
timeout -k 10 420 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-300
timeout -k 10 420 python -u bench.py --gpus 1 --steps 20 --warmup 5 --mode literal --no-cpu-baseline > $T/bench_literal.log 2>&1 || { echo "literal bench failed"; tail -20 $T/bench_literal.log; exit 1; }
tail -1 $T/bench_literal.log | cut -c1-300
echo ALL OK
