#!/bin/bash
# r04a: (1) the split kernel's error distribution on the bench's weights (10 seeds, cfg2-5);
# (2) PMC of the split trunk incl. GRBM_GUI_ACTIVE; (3) the driver's bench command under the host
# sampling profiler (aged window) with the per-ordinal game costs
set -o pipefail
TAG=${1:-r04a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_nn_v2_gpu.py -k concat -x -v --timeout 120 --timeout-method thread > $T/concat_tests.log 2>&1; echo "concat tests rc=$?"; tail -1 $T/concat_tests.log
timeout -k 10 500 python -u tools/split_error_dist.py $T/split_error_dist.json --seeds 10 > $T/split_error_dist.log 2>&1 || { echo "error dist failed"; tail -20 $T/split_error_dist.log; exit 1; }
grep "max over" $T/split_error_dist.log
bash tools/gpu_pmc_r04.sh $TAG/pmc > $T/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $T/pmc.log; exit 1; }
grep -A14 "trunk_kernel" $T/pmc/summary.txt
cd $R
gcc -O2 -shared -fPIC tools/sprof/sprof.c -o $T/sprof.so || exit 1
GZ_SPROF_LIB=$T/sprof.so SPROF_OUT=$T/sprof.out SPROF_START_S=330 SPROF_STOP_S=390 timeout -k 10 580 python -u bench.py --gpus 1 --steps 60 --warmup 5 --no-cpu-baseline > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log | cut -c1-400
python tools/sprof/report.py $T/sprof.out 60 > $T/sprof_report.txt 2>&1 || exit 1
rm -f $T/sprof.so
head -30 $T/sprof_report.txt
echo ALL OK
