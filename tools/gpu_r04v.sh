#!/bin/bash
# r04v (final tree): every GPU test except the long runner ones (r04u ran those) + smoke, then the
# driver's bench command
set -o pipefail
TAG=${1:-r04v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
# heartbeat under gpurun_out (a single test -- the runner's oracle replay -- can run silent for
# minutes); stopped when the script ends
( while sleep 45; do date +%T >> $T/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_r04f.sh $TAG || exit 1
timeout -k 10 900 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-400
echo ALL OK
