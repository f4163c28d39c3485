#!/bin/bash
# r05p: the driver's bench command under the host sampling profiler (tools/sprof, 60 s inside the
# aged window) on the round-5 engine (PGO, AVX2 block spin loops) -- VERDICT r4 item 2's report
set -o pipefail
TAG=${1:-r05p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
gcc -O2 -shared -fPIC tools/sprof/sprof.c -o $T/sprof.so || exit 1
GZ_SPROF_LIB=$T/sprof.so SPROF_OUT=$T/sprof.out SPROF_START_S=300 SPROF_STOP_S=335 timeout -k 10 700 python -u bench.py --gpus 1 --steps 60 --warmup 5 --no-cpu-baseline > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
grep "^{" $T/bench.log | tail -1 | cut -c1-400
python tools/sprof/report.py $T/sprof.out 60 > $T/sprof_report.txt 2>&1 || exit 1
python tools/sprof/report.py $T/sprof.out 80 --lines > $T/sprof_lines.txt 2>&1 || exit 1
rm -f $T/sprof.so
head -40 $T/sprof_report.txt
echo ALL OK
