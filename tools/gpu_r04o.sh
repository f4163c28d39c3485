#!/bin/bash
# r04o: merged head-conv reductions + sequential-heads fallback (lib_hmerge = this product library) vs the previous (lib_cur): cfg2
# timing + stamps, max output difference; then the NN / bench-shape / deep-runner GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04o
mkdir -p $T
cd $R
for n in cur hmerge; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 120 python -u tools/kexp/dump_outputs.py $T/out2_$n.npz > $T/dump2_$n.log 2>&1 || { echo "$n dump failed"; tail -5 $T/dump2_$n.log; exit 1; }
done
python - "$T" <<'PY'
import sys, numpy as np
T = sys.argv[1]
b = np.load(T + "/out2_cur.npz"); o = np.load(T + "/out2_hmerge.npz")
print("cfg2 hmerge vs cur: bit-identical %s, max diff %.3g" % (all(np.array_equal(b[k], o[k]) for k in b.files), max(float(np.abs(b[k] - o[k]).max()) for k in b.files)))
PY
bash tools/gpu_kexp.sh r04o cur hmerge || exit 1
timeout -k 10 700 python -u -m pytest tests/test_nn_gpu.py tests/test_bench_shape_gpu.py tests/test_runner_deep_gpu.py tests/test_nn_v2_gpu.py tests/test_runner_gpu.py -x -v --timeout 300 --timeout-method thread > $T/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $T/tests.log | head; tail -3 $T/tests.log; exit 1; }
tail -1 $T/tests.log
