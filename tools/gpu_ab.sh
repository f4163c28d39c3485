#!/bin/bash
# Same-box A/B of two builds of libgz_nn.so (lib/ vs $B_DIR): forward timing of cfg2/cfg3, twice
# interleaved, plus the NN parity tests on build B.
mkdir -p gpurun_out/ab
B_DIR=${B_DIR:-galvanise_zero_amd/lib_il}
for rep in 1 2; do
  timeout -k 10 200 python tools/kernel_variants.py --configs 2,3 --batches 256,640,1024 --variants default > gpurun_out/ab/a$rep.log 2>&1 || { echo A failed; exit 1; }
  GZ_LIB_DIR=$B_DIR timeout -k 10 200 python tools/kernel_variants.py --configs 2,3 --batches 256,640,1024 --variants default > gpurun_out/ab/b$rep.log 2>&1 || { echo B failed; exit 1; }
done
paste gpurun_out/ab/a1.log gpurun_out/ab/b1.log | awk '{print $1, $4, $5, "A", $6, "B", $18}'
paste gpurun_out/ab/a2.log gpurun_out/ab/b2.log | awk '{print $1, $4, $5, "A", $6, "B", $18}'
GZ_LIB_DIR=$B_DIR timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests_b.log 2>&1 || { echo "B tests failed"; tail -20 gpurun_out/ab/tests_b.log; exit 1; }
tail -1 gpurun_out/ab/tests_b.log
echo ALL OK
