#!/bin/bash
# r04d: deep-config kernel experiment (tools/kexp/build.py full_<name>): cfg4 / cfg5 split outputs
# must be bit-identical to full_base, then kernel timings (tools/kernel_variants.py)
set -o pipefail
TAG=${1:-r04d}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
for n in full_base "$@"; do
  for c in 4 5; do
    GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 180 python -u tools/kexp/dump_outputs.py $T/out_${n}_$c.npz $c > $T/dump_${n}_$c.log 2>&1 || { echo "$n cfg$c dump failed"; tail -5 $T/dump_${n}_$c.log; exit 1; }
  done
done
python - "$T" "$@" <<'PY'
import sys, numpy as np
T = sys.argv[1]
for c in (4, 5):
    b = np.load("%s/out_full_base_%d.npz" % (T, c))
    for n in sys.argv[2:]:
        o = np.load("%s/out_%s_%d.npz" % (T, n, c))
        same = all(np.array_equal(b[k], o[k]) for k in b.files)
        print("cfg%d %s vs full_base: bit-identical %s, max diff %.3g" % (c, n, same, max(float(np.abs(b[k] - o[k]).max()) for k in b.files)))
PY
for rep in 1 2; do
for n in full_base "$@"; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 240 python -u tools/kernel_variants.py --configs 4,5 --batches 256,1024 --reps 5 --precision fp32 --variants default > $T/${n}_$rep.txt 2>&1 || { echo "$n timing failed"; tail -5 $T/${n}_$rep.txt; exit 1; }
  echo "$n rep $rep:"; grep -E 'N=' $T/${n}_$rep.txt
done
done
echo ALL OK
