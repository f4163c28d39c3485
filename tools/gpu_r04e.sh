#!/bin/bash
# r04e: the r04c cfg2 asm-chain experiment, then the r04d deep-config looped-conv experiment
set -o pipefail
bash tools/gpu_r04c.sh r04c asmchain asmchain_nonop > gpurun_out/r04c.log 2>&1; rc=$?
cat gpurun_out/r04c.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04d.sh r04d full_siunroll
