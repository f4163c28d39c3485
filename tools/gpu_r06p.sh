#!/bin/bash
# r06p: the driver's bench command under the host sampling profiler (tools/sprof) inside the aged
# window on the round-6 engine (VERDICT r5 item 4's line report), then the literal-mode line
# (SURVEY 8d "report two modes")
set -o pipefail
TAG=${1:-r06p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
gcc -O2 -shared -fPIC tools/sprof/sprof.c -o $T/sprof.so || exit 1
GZ_SPROF_LIB=$T/sprof.so SPROF_OUT=$T/sprof.out SPROF_START_S=290 SPROF_STOP_S=318 timeout -k 10 700 python -u bench.py --gpus 1 --steps 80 --warmup 5 --no-cpu-baseline > $T/bench_sprof.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_sprof.log; exit 1; }
grep "^{" $T/bench_sprof.log | tail -1 | cut -c1-300
timeout -k 10 200 python tools/sprof/report.py $T/sprof.out 60 > $T/sprof_report.txt 2>&1 || exit 1
timeout -k 10 300 python tools/sprof/report.py $T/sprof.out 80 --lines > $T/sprof_lines.txt 2>&1 || exit 1
rm -f $T/sprof.so $T/sprof.out
head -30 $T/sprof_report.txt
timeout -k 10 700 python -u bench.py --mode literal --no-cpu-baseline > $T/bench_literal.log 2>&1 || { echo "literal bench failed"; tail -20 $T/bench_literal.log; exit 1; }
grep "^{" $T/bench_literal.log | tail -1 | cut -c1-300
