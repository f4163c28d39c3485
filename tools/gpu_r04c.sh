#!/bin/bash
# r04c: kernel experiments (tools/kexp/build.py builds under tools/kexp/lib_<name>): outputs must be
# bit-identical to the base build, then interleaved timing + stamps (tools/gpu_kexp.sh)
set -o pipefail
TAG=${1:-r04c}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
for n in base "$@"; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 120 python -u tools/kexp/dump_outputs.py $T/out_$n.npz > $T/dump_$n.log 2>&1 || { echo "$n dump failed"; tail -5 $T/dump_$n.log; exit 1; }
done
python - "$T" "$@" <<'PY'
import sys, numpy as np
T = sys.argv[1]
b = np.load(T + "/out_base.npz")
for n in sys.argv[2:]:
    o = np.load(T + "/out_%s.npz" % n)
    same = all(np.array_equal(b[k], o[k]) for k in b.files)
    print("%s vs base: bit-identical %s, max diff %.3g" % (n, same, max(float(np.abs(b[k] - o[k]).max()) for k in b.files)))
PY
bash tools/gpu_kexp.sh $TAG base "$@"
