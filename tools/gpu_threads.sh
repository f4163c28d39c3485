#!/bin/bash
# r03t: smoke; engine threads 15 vs 16 on the 16-CPU box (one generation aged, same box)
set -o pipefail
T=gpurun_out/${1:-r03t}
mkdir -p $T


for th in ${THREADS:-15 16}; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --age-games 1 --threads $th --no-cpu-baseline > $T/bench_t$th.log 2>&1 || { echo "bench t$th failed"; tail -5 $T/bench_t$th.log; exit 1; }
  tail -1 $T/bench_t$th.log | cut -c1-200
done
echo ALL OK
