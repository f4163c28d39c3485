#!/bin/bash
# r05c: errors vs the oracle after the im2col swizzle fix (large boards, v2 files, initial-conv widths)
set -o pipefail
TAG=${1:-r05c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 500 python -u tools/large_board_errors.py > $T/errors.log 2>&1 || { echo "errors script failed"; tail -20 $T/errors.log; exit 1; }
cat $T/errors.log
