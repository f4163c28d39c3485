#!/bin/bash
# pools per engine thread (16 threads, one generation aged, same box)
set -o pipefail
T=gpurun_out/${1:-pools}
mkdir -p $T
for p in ${POOLS:-2 3}; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --age-games 1 --pools $p --no-cpu-baseline > $T/bench_p$p.log 2>&1 || { echo "bench p$p failed"; tail -5 $T/bench_p$p.log; exit 1; }
  tail -1 $T/bench_p$p.log | cut -c1-200
done
echo ALL OK
