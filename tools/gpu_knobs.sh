#!/bin/bash
# Short-window A/B of bench knobs (same box): default, 16 engine threads, bigger launch batches.
set -o pipefail
mkdir -p gpurun_out/knobs
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 4000 --no-cpu-baseline "$@" > gpurun_out/knobs/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/knobs/$tag.log; exit 1; }; tail -1 gpurun_out/knobs/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', round(d['value']), round(d['games_per_sec'],2), d['config']['threads_per_gpu'], round(d['gpu_busy_frac'],3), r['kernel'], round(r['frac'],3))"; }
run base
run t16 --threads 16
run big --min-launch-rows 2048 --max-launch-wait-us 6000
run base2
echo ALL OK
