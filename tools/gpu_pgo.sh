#!/bin/bash
# PGO training run on the GPU box: the bench's command (aged window) on the instrumented engine
# (galvanise_zero_amd/lib_pgogen, built here by `make -C galvanise_zero_amd/csrc PGO=gen
# LIBDIR=$PWD/galvanise_zero_amd/lib_pgogen`); gcc writes the profiles to gpurun_out/pgo_gen, which
# tools/pgo_install.sh copies to galvanise_zero_amd/csrc/pgo with the sources manifest.
set -o pipefail
TAG=${1:-pgo}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
rm -rf $R/gpurun_out/pgo_gen
GZ_LIB_DIR=$R/galvanise_zero_amd/lib_pgogen timeout -k 10 540 python -u bench.py --gpus 1 --steps 5 --warmup 2 --age-games 3 --age-seconds 240 --no-cpu-baseline > $T/pgo_bench.log 2>&1 || { echo "pgo bench failed"; tail -5 $T/pgo_bench.log; exit 1; }
tail -1 $T/pgo_bench.log | cut -c1-200
find $R/gpurun_out/pgo_gen -name "*.gcda" | wc -l
