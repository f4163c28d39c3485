#!/bin/bash
# r02d: the GPU box's CPU share, then the host engine probe (no GPU): 1 / 15 / 31 threads, child
# mirror on / off
set -o pipefail
T=gpurun_out/r02d
mkdir -p $T
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > $T/cpu.txt 2>&1
cat $T/cpu.txt
for b in engine_mirror engine_nomirror; do
  for th in 1 15 31; do
    timeout -k 10 200 ./tools/$b.bin 256 6000 800 $th 1000 > $T/${b}_t${th}.txt 2>&1 || { echo "$b $th failed"; exit 1; }
    echo "$b t$th: $(tail -n 1 $T/${b}_t${th}.txt)"
  done
done
echo ALL OK
