#!/bin/bash
# r05lr: launch batching -- the driver's bench (default aging, 20 steps, no CPU leg) with
# --min-launch-rows 1024 (the default) and 2048, the same box back to back
set -o pipefail
TAG=${1:-r05lr}
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/$TAG
mkdir -p $T
cd $R
for m in 1024 2048; do
  timeout -k 10 560 python -u bench.py --min-launch-rows $m --no-cpu-baseline > $T/bench_m$m.log 2>&1 || { echo "m$m failed"; tail -5 $T/bench_m$m.log; exit 1; }
  grep "^{" $T/bench_m$m.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('min_launch_rows $m', 'value %.0f games/s %.1f busy %.3f idle %.3f kernel_ms %.4f rows %.1f frac %.4f' % (d['value'], d['games_per_sec'], d['gpu_busy_frac'], d.get('engine_idle_frac', -1), r['avg_kernel_ms'], r['rows_per_launch'], r['frac']))"
done
