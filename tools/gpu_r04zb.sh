#!/bin/bash
# r04zb: the driver's bench command on the final tree (default settings)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04zb
mkdir -p $T
cd $R
( while sleep 45; do date +%T >> $T/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 840 python -u bench.py > $T/bench.log 2>&1 || { echo "bench failed"; tail -5 $T/bench.log; exit 1; }
grep "^{" $T/bench.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('value', round(d['value']), 'games/s', d.get('games_per_sec'), 'busy', round(d['gpu_busy_frac'],3), 'kernel', r['kernel'], 'ms', round(r['avg_kernel_ms'],4), 'frac', round(r['frac'],4), 'cpu', d['cpu_baseline']['value'])"
echo ALL OK
