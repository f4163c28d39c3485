#!/bin/bash
# queue helper: re-submits only when gpurun reports that nothing ran (no slot / no box)
OUT=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  if grep -q "nothing was charged\|no free box right now\|while being prepared; retry\|backing off" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then sleep 150; continue; fi
  break
done
