#!/usr/bin/env python3
"""Per-kernel register/occupancy table of mirbft_amd/csrc/kernels.hip (hipcc
-Rpass-analysis=kernel-resource-usage), to check spills and occupancy after a change."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "mirbft_amd/csrc/kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-c", src,
       "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = cur.split("(")[0]
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
for k, v in rows.items():
    print(f"{k:52s} VGPR={v.get('VGPRs'):>4} spillV={v.get('VGPRs Spill')} spillS={v.get('SGPRs Spill')} "
          f"occ={v.get('Occupancy [waves/SIMD]')}")
