#!/bin/bash
# Register / spill / LDS usage of every kernel of libgz_nn (device-only compile, no GPU needed).
for tu in gz_nn trunk_f64 trunk_f128 trunk_f256 trunk_f64_v2 trunk_f128_v2; do
cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-parameter -I/root/repo/include \
  --cuda-device-only -c /root/repo/galvanise_zero_amd/csrc/nn/$tu.hip -o /tmp/gz_dev_$tu.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re, subprocess
cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip(); rows[cur] = {}
        continue
    m = re.search(r"remark: ([A-Za-z ]+): (\d+)", line)
    if m and cur: rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if "trunk" in k or "heads" in k:
        print("%-60s VGPR %4s AGPR %4s spillV %3s" % (k[:60], v.get("VGPRs"), v.get("AGPRs"), v.get("VGPRs Spill")))
'
done
