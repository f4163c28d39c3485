#!/bin/bash
# A/B of the forward kernel: the in-tree library (new) against tools/ab_old_lib (previous commit),
# alternating, per config at 1,024 rows.  Usage: bash tools/ab_forward.sh <tag> [configs]
set -o pipefail
TAG=${1:-ab}; CFGS=${2:-"1 2 3 4 5"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG; cd $R
for round in 1 2; do
  for c in $CFGS; do
    echo "== round $round cfg$c new"; timeout -k 10 120 python -u tools/time_forward.py --config $c --rows 1024 --reps 15 || exit 1
    echo "== round $round cfg$c old"; GZ_LIB_DIR=$R/tools/ab_old_lib timeout -k 10 120 python -u tools/time_forward.py --config $c --rows 1024 --reps 15 || exit 1
  done
done 2>&1 | tee $R/gpurun_out/$TAG/ab.txt
