#!/bin/bash
# r05kr: variant 23 with a 2-stage weight ring (tools/kexp/lib_h2ring2, -DGZ_H2_RING_VGPRS=96)
# against the default 4-stage ring: identity (21 vs 23 inside the experimental library) and the
# forward at 1,024 rows, alternating; and with the lane-swapped epilogue stores (lib_h2swap,
# -DGZ_STORE_SWAP=1)
set -o pipefail
TAG=${1:-r05kr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
GZ_LIB_DIR=$R/tools/kexp/lib_h2ring2 timeout -k 10 200 python -u tools/variant_diff.py 21 23 > $T/diff_ring2.txt 2>&1 || { tail -5 $T/diff_ring2.txt; exit 1; }
cat $T/diff_ring2.txt
GZ_LIB_DIR=$R/tools/kexp/lib_h2swap timeout -k 10 200 python -u tools/variant_diff.py 21 23 > $T/diff_swap.txt 2>&1 || { tail -5 $T/diff_swap.txt; exit 1; }
cat $T/diff_swap.txt
for round in 1 2 3; do
  echo "== round $round ring 4 (default)"; timeout -k 10 120 python -u tools/time_forward.py --config 2 --rows 1024 --reps 15 --precision fp32 || exit 1
  echo "== round $round ring 2"; GZ_LIB_DIR=$R/tools/kexp/lib_h2ring2 timeout -k 10 120 python -u tools/time_forward.py --config 2 --rows 1024 --reps 15 --precision fp32 || exit 1
  echo "== round $round store swap"; GZ_LIB_DIR=$R/tools/kexp/lib_h2swap timeout -k 10 120 python -u tools/time_forward.py --config 2 --rows 1024 --reps 15 --precision fp32 || exit 1
done 2>&1 | tee $T/ab_ring.txt
