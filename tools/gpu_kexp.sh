#!/bin/bash
# Diagnostic builds (tools/kexp/build.py) timed on one box, twice interleaved: cfg2 fp32 variant 21
# forward times and per-phase stamps.  usage: bash tools/gpu_kexp.sh TAG name...
set -o pipefail
TAG=$1; shift
T=gpurun_out/$TAG
mkdir -p $T
for rep in 1 2; do
for n in "$@"; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 120 python -u tools/kernel_variants.py --configs 2 --batches 512,1024,2048 --reps 20 --precision fp32 --variants 21 > $T/${n}_$rep.txt 2>&1 || { echo "$n failed"; tail -5 $T/${n}_$rep.txt; exit 1; }
  echo "$n rep $rep: $(grep -E 'N=' $T/${n}_$rep.txt | awk '{printf "%s %s ms | ", $6, $7}')"
done
done
for n in "$@"; do
  GZ_LIB_DIR=tools/kexp/lib_$n timeout -k 10 120 python -u tools/kernel_breakdown.py --precision fp32 --variants 21 --batches 1024 --blocks 0,6 > $T/${n}_stamps.txt 2>&1 || { echo "$n stamps failed"; tail -5 $T/${n}_stamps.txt; exit 1; }
  echo "$n: $(grep -E 'stamps|fixed' $T/${n}_stamps.txt | tr '\n' ' ')"
done
echo ALL OK
