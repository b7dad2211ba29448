#!/usr/bin/env python3
"""Per-kernel resource usage of encode.hip (hipcc -Rpass-analysis) as a table."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "airs-compression_amd/csrc/encode.hip"
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
                      "-Iairs-compression_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rows.items():
    if filt in k:
        print(f"{k[:60]:60s} vgpr={v.get('VGPRs')} sgpr={v.get('TotalSGPRs')} occ={v.get('Occupancy [waves/SIMD]')} "
              f"lds={v.get('LDS Size [bytes/block]')} sspill={v.get('SGPRs Spill')} vspill={v.get('VGPRs Spill')}")
