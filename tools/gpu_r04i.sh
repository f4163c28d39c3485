#!/bin/bash
# r04i: ring-depth experiments (tools/kexp ring6 / ring12 vs base), then r04h (PMC + bench)
set -o pipefail
bash tools/gpu_r04c.sh r04i ring6 ring12 > gpurun_out/r04i.log 2>&1; rc=$?
cat gpurun_out/r04i.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04h.sh r04h
