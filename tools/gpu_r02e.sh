#!/bin/bash
# r02e: steady-state engine probe on the box's CPUs (1 and 15 threads, 32 games per thread), then
# the driver's bench command (CPU share from the cgroup quota, fp32-accuracy net not yet default)
set -o pipefail
T=gpurun_out/r02e
mkdir -p $T
for th in 1 15; do
  timeout -k 10 240 ./tools/engine_new.bin 32 60000 800 $th 1000 > $T/engine_t${th}.txt 2>&1 || { echo "probe $th failed"; exit 1; }
  echo "t$th: $(tail -n 1 $T/engine_t${th}.txt)"
done
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $T/bench.log 2>&1 || { echo "bench failed"; tail -20 $T/bench.log; exit 1; }
tail -1 $T/bench.log
echo ALL OK
