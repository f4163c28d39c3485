#!/bin/bash
# r06d: reversi (BASELINE cfg3) bench regime on the GPU box: spin / exit counters (GZ_SPIN_STATS),
# a few dumps of long-spinning roots (GZ_SPIN_DUMP) and the host sampling profiler over the timed steps
set -o pipefail
TAG=${1:-r06d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
gcc -O2 -shared -fPIC tools/sprof/sprof.c -o $T/sprof.so || exit 1
GZ_SPIN_STATS=1 GZ_SPIN_DUMP=1000000 GZ_SPROF_LIB=$T/sprof.so SPROF_OUT=$T/sprof.out SPROF_START_S=250 SPROF_STOP_S=330 \
  timeout -k 10 900 python -u bench.py --config 3 --age-seconds 240 --steps 8 --warmup 1 --no-cpu-baseline > $T/bench_cfg3.log 2>&1 || { echo "bench failed"; tail -20 $T/bench_cfg3.log; exit 1; }
grep "^{" $T/bench_cfg3.log | tail -1 | cut -c1-400
grep "gz spin stats" $T/bench_cfg3.log | tail -1
timeout -k 10 300 python tools/sprof/report.py $T/sprof.out 50 > $T/sprof_report.txt 2>&1 || exit 1
rm -f $T/sprof.so
head -30 $T/sprof_report.txt
