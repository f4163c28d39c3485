#!/bin/bash
# r03g: looped vs unrolled conv (same box), stamps, variant timings (fp32 cfg2/3/5, bf16 cfg2-5)
set -o pipefail
T=gpurun_out/${1:-r03g}
mkdir -p $T
bash tools/gpu_kexp.sh $1/kexp base unroll || exit 1
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3 --batches 256,512,1024,2048 --reps 20 --precision fp32 --variants default,11,21 > $T/variants_fp32.txt 2>&1 || { echo "variants failed"; tail -5 $T/variants_fp32.txt; exit 1; }
grep "N= 1024\|N= 2048" $T/variants_fp32.txt
timeout -k 10 300 python -u tools/kernel_variants.py --configs 5 --batches 256,1024,2560 --reps 5 --precision fp32 --variants default > $T/variants_cfg5_fp32.txt 2>&1 || { echo "cfg5 fp32 failed"; tail -5 $T/variants_cfg5_fp32.txt; exit 1; }
cat $T/variants_cfg5_fp32.txt
GZ_NO_GEMM_HEADS=1 timeout -k 10 300 python -u tools/kernel_variants.py --configs 5 --batches 256,1024,2560 --reps 5 --precision fp32 --variants default > $T/variants_cfg5_fp32_nogemm.txt 2>&1 || { echo "cfg5 fp32 nogemm failed"; exit 1; }
cat $T/variants_cfg5_fp32_nogemm.txt
timeout -k 10 300 python -u tools/kernel_variants.py --configs 2,3,4,5 --batches 256,1024 --reps 10 --precision bf16 --variants default > $T/variants_bf16.txt 2>&1 || { echo "variants bf16 failed"; tail -5 $T/variants_bf16.txt; exit 1; }
grep "N= 1024" $T/variants_bf16.txt
echo ALL OK
