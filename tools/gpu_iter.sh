mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python tools/kernel_variants.py --configs 1,2 --batches 256,512,1024,4096 > gpurun_out/kv.log 2>&1 || { echo kv failed; exit 1; }
timeout -k 10 200 python tools/kernel_breakdown.py --variants 12,21 --batches 256,512,1024 > gpurun_out/breakdown.log 2>&1 || { echo bd failed; exit 1; }
echo ALL OK
