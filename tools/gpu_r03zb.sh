#!/bin/bash
# r03zb: host sampling profile of the driver's bench command on the final engine, in the aged
# window (three generations: samples from 330 s to 390 s, a 120-step window), report on the box
set -o pipefail
TAG=${1:-r03zb}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
gcc -O2 -shared -fPIC tools/sprof/sprof.c -o $T/sprof.so || exit 1
GZ_SPROF_LIB=$T/sprof.so SPROF_OUT=$T/sprof.out SPROF_START_S=330 SPROF_STOP_S=390 timeout -k 10 560 python -u bench.py --gpus 1 --steps 120 --warmup 5 --no-cpu-baseline > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-300
python tools/sprof/report.py $T/sprof.out 60 > $T/sprof_report.txt 2>&1 || exit 1
rm -f $T/sprof.so
head -45 $T/sprof_report.txt
echo ALL OK
