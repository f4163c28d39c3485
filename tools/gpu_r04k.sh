#!/bin/bash
# r04k: quad-layout dense heads (tools/kexp/lib_heads4 = the product library) vs the previous heads
# (lib_base): bit-identity + timing + stamps on cfg2; then cfg5 / cfg4 short aged benches under
# rocprofv3 --kernel-trace --stats (heads share of GPU time, trunk frac)
set -o pipefail
bash tools/gpu_r04c.sh r04k heads4 > gpurun_out/r04k.log 2>&1; rc=$?
cat gpurun_out/r04k.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_cfg_aged.sh r04k "5 4" 60
