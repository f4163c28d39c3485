#!/bin/bash
# r04y (final tree): every GPU test except the long runner ones + smoke, with a heartbeat
set -o pipefail
TAG=${1:-r04y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 45; do date +%T >> $T/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_r04f.sh $TAG || exit 1
bash tools/gpu_r04u.sh ${TAG}_long > $T/long.log 2>&1 || { echo "long tests failed"; tail -20 $T/long.log; exit 1; }
tail -4 $T/long.log
echo ALL OK
