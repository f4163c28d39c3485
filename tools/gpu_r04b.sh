#!/bin/bash
# r04b: (1) the new GPU tests of this round (live verification window aged to the bench's regime,
# roll timeout, runner re-create memory, the deep configs' full nets through the runner vs the
# oracle, concat head); (2) the PGO training run: the bench's command on an instrumented engine
# (galvanise_zero_amd/lib_pgogen, `make PGO=gen LIBDIR=...`) whose gcc profile lands in
# gpurun_out/pgo_gen (copied to galvanise_zero_amd/csrc/pgo for the -fprofile-use build)
set -o pipefail
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
timeout -k 10 900 python -u -m pytest tests/test_runner_verify_gpu.py tests/test_runner_roll_gpu.py tests/test_runner_deep_gpu.py tests/test_nn_v2_gpu.py -k "aged or timeout or recreate or deep or concat" -v -s --timeout 600 --timeout-method thread > $T/tests.log 2>&1; echo "tests rc=$?"
grep -E "PASSED|FAILED|ERROR|passed|failed" $T/tests.log | tail -15
grep -E "^\{|verify verified|cycle|short-timeout|identical to the oracle" $T/tests.log | tail -12
GZ_LIB_DIR=$R/galvanise_zero_amd/lib_pgogen timeout -k 10 420 python -u bench.py --gpus 1 --steps 5 --warmup 2 --age-games 3 --age-seconds 200 --no-cpu-baseline > $T/pgo_bench.log 2>&1 || { echo "pgo bench failed"; tail -5 $T/pgo_bench.log; exit 1; }
tail -1 $T/pgo_bench.log | cut -c1-200
find $R/gpurun_out/pgo_gen -name "*.gcda" | wc -l
echo ALL OK
