#!/bin/bash
# r04g: dense-heads experiments on the cfg2 split kernel (tools/kexp: headsunroll bit-identical to
# base, noheads = the heads' cost), then variant 21 vs 22 (two wave groups) with the product library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_r04c.sh r04g headsunroll || exit 1
timeout -k 10 180 python -u tools/kernel_variants.py --configs 2 --batches 512,1024,2048 --reps 20 --precision fp32 --variants 21,22 > gpurun_out/r04g/v21_v22.txt 2>&1 || { echo "variants failed"; tail -5 gpurun_out/r04g/v21_v22.txt; exit 1; }
cat gpurun_out/r04g/v21_v22.txt
GZ_LIB_DIR=tools/kexp/lib_noheads timeout -k 10 120 python -u tools/kernel_breakdown.py --precision fp32 --variants 21 --batches 1024 --blocks 0,6 > gpurun_out/r04g/noheads_stamps.txt 2>&1 || { echo "noheads failed"; exit 1; }
echo "noheads: $(grep -E 'stamps|fixed' gpurun_out/r04g/noheads_stamps.txt | tr '\n' ' ')"
echo ALL OK
