#!/bin/bash
# Installs the profiles of a PGO training run (tools/gpu_pgo.sh) into galvanise_zero_amd/csrc/pgo,
# keyed by the objects' absolute paths as gcc looks them up, with the manifest of the engine sources
# they were recorded on (csrc/Makefile uses them only while that manifest matches), then rebuilds.
set -e
R=$(cd $(dirname $0)/.. && pwd)
P=$R/galvanise_zero_amd/csrc/pgo
SRC=$R/gpurun_out/pgo_gen$R/galvanise_zero_amd/build/engine
[ -d "$SRC" ] || { echo "no profiles under $SRC"; exit 1; }
rm -rf $P && mkdir -p $P$R/galvanise_zero_amd/build/engine
cp $SRC/*.gcda $P$R/galvanise_zero_amd/build/engine/
(cd $R/galvanise_zero_amd && sha256sum $(ls csrc/engine/*.cpp csrc/engine/*.h | LC_ALL=C sort)) > $P/sources.sha256
make -C $R/galvanise_zero_amd/csrc -j8 PGO=use
