#!/bin/bash
# r04x: variant 21 vs 24 inside the bench (same box, back to back, 200 s aging each): the kernel's
# average launch time under the engine threads' host load decides the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$R/gpurun_out/r04x
mkdir -p $T
cd $R
for v in 24 21; do
  GZ_KERNEL_VARIANT=$v timeout -k 10 560 python -u bench.py --no-cpu-baseline --age-seconds 200 --steps 12 --warmup 3 > $T/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $T/bench_$v.log; exit 1; }
  grep "^{" $T/bench_$v.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('variant $v', round(d['value']), 'busy', round(d['gpu_busy_frac'],3), 'kernel', r['kernel'], 'ms', round(r['avg_kernel_ms'],4), 'rows', round(r['rows_per_launch'],1), 'frac', round(r['frac'],4))"
done
echo ALL OK
