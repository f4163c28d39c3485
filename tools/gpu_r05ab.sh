#!/bin/bash
# r05ab: variant 23 (default) against 21 inside the bench, the same box back to back (aged 150 s,
# 10 steps each, no CPU leg): the dominant kernel's event-timed launch time per variant
set -o pipefail
TAG=${1:-r05ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
( while sleep 60; do date +%T >> $T/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in 21 23; do
  GZ_KERNEL_VARIANT=$v timeout -k 10 400 python -u bench.py --age-seconds 150 --steps 10 --warmup 3 --no-cpu-baseline > $T/bench_v$v.log 2>&1 || { echo "v$v failed"; tail -5 $T/bench_v$v.log; exit 1; }
  grep "^{" $T/bench_v$v.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('variant $v', r['kernel'], 'avg_kernel_ms %.4f rows %.1f frac %.4f value %.0f busy %.3f' % (r['avg_kernel_ms'], r['rows_per_launch'], r['frac'], d['value'], d['gpu_busy_frac']))"
done
