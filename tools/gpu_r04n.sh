#!/bin/bash
# r04n: two-phase dense heads + LDS-DMA lo copy-in (+ raw barrier after the copy-out): cfg4 / cfg5
# outputs bit-identical to the previous build (lib_full_prev) and timed; cfg2 likewise (lib_conv0 =
# the previous product library, lib_cur = this one)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04n
mkdir -p $T
cd $R
bash tools/gpu_r04d.sh r04n full_prev || exit 1
for n in conv0 cur; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 120 python -u tools/kexp/dump_outputs.py $T/out2_$n.npz > $T/dump2_$n.log 2>&1 || { echo "$n dump failed"; tail -5 $T/dump2_$n.log; exit 1; }
done
python - "$T" <<'PY'
import sys, numpy as np
T = sys.argv[1]
b = np.load(T + "/out2_conv0.npz"); o = np.load(T + "/out2_cur.npz")
print("cfg2 cur vs conv0: bit-identical %s, max diff %.3g" % (all(np.array_equal(b[k], o[k]) for k in b.files), max(float(np.abs(b[k] - o[k]).max()) for k in b.files)))
PY
bash tools/gpu_kexp.sh r04n conv0 cur
